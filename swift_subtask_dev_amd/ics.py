"""Synthetic initial conditions for the benchmark configurations and tests.

The real SWIFT ICs (glassCube_64.hdf5, EAGLE_ICs_6.hdf5, SmallCosmoVolume)
are `wget`-only and unavailable offline; these generators build
inputs of the same shape from recipes cited per function. Every generator is
deterministic (numpy PCG64 with a recorded seed).
"""
from __future__ import annotations

import numpy as np

from . import abi

GAMMA = 5.0 / 3.0


def _rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


def perturbed_lattice(n: int, box: float = 1.0, pert: float = 0.1, seed: int = 0x5EED):
    """n^3 lattice points (i+0.5)/n*box, each coordinate displaced by
    uniform(-0.5, 0.5)*pert/n*box (tests/test27cells.c make_cell, -d pert)."""
    rng = _rng(seed)
    g = (np.arange(n) + 0.5) / n
    x, y, z = np.meshgrid(g, g, g, indexing="ij")
    pos = np.stack([x.ravel(), y.ravel(), z.ravel()], axis=1)
    pos = pos + rng.uniform(-0.5, 0.5, size=pos.shape) * pert / n
    pos = np.mod(pos * box, box)
    return pos


def sedov_slabs(n: int, nslab: int, eta: float = 1.2348, pert: float = 0.1,
                seed: int = 0x5EED, rho0: float = 1.0, P0: float = 1.0e-6, E0: float = 1.0,
                n_inject: int = 15) -> np.ndarray:
    """`nslab` unit Sedov cubes side by side along x: a periodic (nslab, 1, 1)
    box of (n*nslab) x n x n perturbed-lattice particles, the blast in the
    centre of the whole box. nslab = 1 is exactly sedov_box(n)'s recipe.
    Used for the weak-scaling decomposition (one unit slab per GPU)."""
    rng = _rng(seed)
    N = n ** 3 * nslab
    p = abi.new_parts(N)
    gx = (np.arange(n * nslab) + 0.5) / n
    g = (np.arange(n) + 0.5) / n
    # chunked fill keeps peak host memory at ~one slab of temporaries
    for s in range(nslab):
        x, y, z = np.meshgrid(gx[s * n:(s + 1) * n], g, g, indexing="ij")
        pos = np.stack([x.ravel(), y.ravel(), z.ravel()], axis=1)
        pos += rng.uniform(-0.5, 0.5, size=pos.shape) * pert / n
        pos[:, 0] = np.mod(pos[:, 0], nslab)
        pos[:, 1:] = np.mod(pos[:, 1:], 1.0)
        p["x"][s * n ** 3:(s + 1) * n ** 3] = pos
    p["id"] = np.arange(1, N + 1)
    m = rho0 * nslab / N
    p["mass"] = m
    p["h"] = eta / n
    p["u"] = P0 / (rho0 * (GAMMA - 1.0))
    c = np.array([0.5 * nslab, 0.5, 0.5])
    r2 = ((p["x"] - c) ** 2).sum(axis=1)
    idx = np.argpartition(r2, n_inject)[:n_inject]
    p["u"][idx] = E0 / (n_inject * m)
    p["time_bin"] = 1
    p["visc_alpha"] = 0.1
    p["min_ngb_time_bin"] = abi.NUM_TIME_BINS + 1
    return p


def sedov_box(n: int, eta: float = 1.2348, pert: float = 0.1, seed: int = 0x5EED,
              velocity: str = "zero", rho0: float = 1.0, P0: float = 1.0e-6, E0: float = 1.0,
              n_inject: int = 15) -> np.ndarray:
    """SedovBlast_3D-like periodic unit box of n^3 gas particles
    (examples/HydroTests/SedovBlast_3D/makeIC.py: rho0=1, P0=1e-6, E0=1 into
    the 15 particles closest to the centre; sedov.yml resolution_eta=1.2348).
    The glass file is replaced by a 10%-perturbed lattice; h = eta * L / n.
    velocity: "zero" (Sedov) or "divergent" (v = x - 0.5, test27cells.c:138)."""
    N = n ** 3
    pos = perturbed_lattice(n, 1.0, pert, seed)
    p = abi.new_parts(N)
    p["id"] = np.arange(1, N + 1)
    p["x"] = pos
    m = rho0 * 1.0 / N
    p["mass"] = m
    p["h"] = eta / n
    u = np.full(N, P0 / (rho0 * (GAMMA - 1.0)), dtype=np.float64)
    r = np.sqrt(((pos - 0.5) ** 2).sum(axis=1))
    idx = np.argsort(r, kind="stable")[:n_inject]
    u[idx] = E0 / (n_inject * m)
    p["u"] = u
    if velocity == "divergent":
        p["v"] = (pos - 0.5).astype(np.float32)
    elif velocity == "random":
        p["v"] = _rng(seed + 1).uniform(-0.05, 0.05, size=(N, 3)).astype(np.float32)
    p["time_bin"] = 1
    p["visc_alpha"] = 0.1
    p["min_ngb_time_bin"] = abi.NUM_TIME_BINS + 1
    return p


def flow_box(n: int, seed: int = 64) -> np.ndarray:
    """A periodic n^3 box in a converging, shearing flow with a lumpy internal
    energy, smoothing lengths off target (the ghost iterates) and switch
    state as an earlier step leaves it (div_v_previous_step, alphas): every
    term of the SPHENIX chain is live -- the artificial viscosity of
    approaching pairs (mu_ij < 0), the diffusion, the viscosity switch
    (hydro_iact.h:130-609, hydro.h:714-934). All particles active."""
    rng = _rng(seed)
    p = sedov_box(n, pert=0.3, seed=seed)
    N = len(p)
    x = p["x"]
    v = -2.0 * (x - 0.5) + rng.normal(0.0, 0.3, (N, 3))
    v[:, 0] += 0.8 * np.sin(2 * np.pi * x[:, 1])  # shear: rot_v != 0
    p["v"] = v.astype(np.float32)
    p["u"] = (1.0 + 0.5 * np.sin(2 * np.pi * x[:, 0]) * np.cos(2 * np.pi * x[:, 2])
              + 0.2 * rng.uniform(size=N)).astype(np.float32)
    p["h"] *= rng.uniform(0.85, 1.2, N)
    p["div_v_previous_step"] = rng.uniform(-4.0, 4.0, N)
    p["visc_alpha"] = rng.uniform(0.0, 1.5, N)
    p["diff_alpha"] = rng.uniform(0.0, 0.8, N)
    return p


def clustered_box(n_bg: int, n_clumps: int = 8, per_clump: int = 4096, seed: int = 6,
                  eta: float = 1.2348) -> np.ndarray:
    """EAGLE_6-like stand-in: a uniform background lattice plus
    Plummer-sphere clumps, so smoothing lengths span more than an order of
    magnitude after the ghost converges them. Periodic unit box."""
    rng = _rng(seed)
    bg = perturbed_lattice(n_bg, 1.0, 0.3, seed)
    clumps = []
    for _ in range(n_clumps):
        c = rng.uniform(0.15, 0.85, 3)
        a = rng.uniform(0.01, 0.03)
        # Plummer radii: r = a / sqrt(u^(-2/3) - 1)
        uu = rng.uniform(0.05, 0.9, per_clump)
        rr = a / np.sqrt(uu ** (-2.0 / 3.0) - 1.0)
        d = rng.normal(size=(per_clump, 3))
        d /= np.linalg.norm(d, axis=1)[:, None]
        clumps.append(np.mod(c + d * rr[:, None], 1.0))
    pos = np.concatenate([bg] + clumps)
    N = len(pos)
    p = abi.new_parts(N)
    p["id"] = np.arange(1, N + 1)
    p["x"] = pos
    p["mass"] = 1.0 / N
    p["h"] = eta / n_bg  # the ghost adapts it
    p["u"] = 1.0
    p["v"] = rng.normal(scale=0.01, size=(N, 3)).astype(np.float32)
    p["time_bin"] = 1
    p["visc_alpha"] = 0.1
    return p


def make_cell(n: int, offset, size: float, h: float, density: float, first_id: int,
              pert: float, vel: str, h_pert: float, rng: np.random.Generator,
              shuffle: bool = True) -> np.ndarray:
    """tests/test27cells.c make_cell:95-211 — n^3 particles on a (perturbed)
    lattice in one cell; h = size*h*U(1, h_pert)/n; mass = rho V / count;
    velocity fields zero / random / divergent (about 1.5*size) / rotating."""
    count = n ** 3
    p = abi.new_parts(count)
    k = 0
    pos = np.empty((count, 3))
    for ix in range(n):
        for iy in range(n):
            for iz in range(n):
                r = rng.uniform(-0.5, 0.5, 3) * pert
                pos[k] = [offset[0] + size * (ix + 0.5 + r[0]) / n,
                          offset[1] + size * (iy + 0.5 + r[1]) / n,
                          offset[2] + size * (iz + 0.5 + r[2]) / n]
                k += 1
    p["x"] = pos
    if vel == "zero":
        p["v"] = 0.0
    elif vel == "random":
        p["v"] = rng.uniform(-0.05, 0.05, (count, 3)).astype(np.float32)
    elif vel == "divergent":
        p["v"] = (pos - 1.5 * size).astype(np.float32)
    elif vel == "rotating":
        v = np.zeros((count, 3))
        v[:, 0] = pos[:, 1]
        v[:, 1] = -pos[:, 0]
        p["v"] = v.astype(np.float32)
    if h_pert:
        p["h"] = size * h * rng.uniform(1.0, h_pert, count) / n
    else:
        p["h"] = size * h / n
    p["id"] = np.arange(first_id + 1, first_id + count + 1)
    p["mass"] = density * size ** 3 / count
    p["time_bin"] = 1
    if shuffle:
        p[:] = p[rng.permutation(count)]
    return p


def uniform_gravity_box(n: int, epsilon: float = 0.001, seed: int = 256) -> np.ndarray:
    """GravityTests uniform DM box stand-in (examples/GravityTests/Gravity_glass:
    L=1, rho=1; uniform_DM_box.yml comoving_softening 0.001): n^3 uniform
    random gparts of mass 1/N."""
    rng = _rng(seed)
    N = n ** 3
    g = abi.new_gparts(N)
    g["id_or_neg_offset"] = np.arange(1, N + 1)
    g["x"] = rng.uniform(0.0, 1.0, (N, 3))
    g["mass"] = 1.0 / N
    g["epsilon"] = epsilon
    g["time_bin"] = 1
    g["type"] = 1
    return g


def leaf_cells(gparts: np.ndarray, cdim: int, box: float = 1.0):
    """Sort gparts into a cdim^3 grid of leaves; returns (sorted gparts,
    leaves[start,count], cell coords). Used for P2P over neighbouring leaves."""
    x = np.mod(gparts["x"], box)
    c = np.minimum((x / (box / cdim)).astype(np.int64), cdim - 1)
    key = (c[:, 0] * cdim + c[:, 1]) * cdim + c[:, 2]
    order = np.argsort(key, kind="stable")
    g = gparts[order].copy()
    key = key[order]
    counts = np.bincount(key, minlength=cdim ** 3)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    leaves = np.zeros(cdim ** 3, dtype=abi.LEAF_DTYPE)
    leaves["start"] = starts
    leaves["count"] = counts
    return g, leaves


def neighbour_pairs(cdim: int, periodic: bool = True, truncated: int = 0):
    """CSR list: every leaf interacts with itself and its 26 neighbours."""
    offs = []
    pairs = []
    for cx in range(cdim):
        for cy in range(cdim):
            for cz in range(cdim):
                offs.append(len(pairs))
                seen = set()
                for dx in (-1, 0, 1):
                    for dy in (-1, 0, 1):
                        for dz in (-1, 0, 1):
                            nx, ny, nz = cx + dx, cy + dy, cz + dz
                            if periodic:
                                nx, ny, nz = nx % cdim, ny % cdim, nz % cdim
                            elif not (0 <= nx < cdim and 0 <= ny < cdim and 0 <= nz < cdim):
                                continue
                            j = (nx * cdim + ny) * cdim + nz
                            if j in seen:
                                continue
                            seen.add(j)
                            pairs.append((j, truncated))
    offs.append(len(pairs))
    arr = np.zeros(len(pairs), dtype=abi.LEAF_PAIR_DTYPE)
    if pairs:
        arr["j"] = [p[0] for p in pairs]
        arr["truncated"] = [p[1] for p in pairs]
    return np.asarray(offs, dtype=np.int32), arr


def gravity_tree(gparts: np.ndarray, cdim: int, split_size: int = 64, box: float = 1.0,
                 max_depth: int = 12):
    """SWIFT-like cell tree (space_split, src/space_split.c): a cdim^3 grid of
    top-level cells, each split into octants while it holds more than
    split_size gparts. Returns (gparts sorted so that every cell is a
    contiguous range, cells as abi.GCell-compatible records, top-level cell
    indices). Empty octants get no cell (progeny -1)."""
    x = np.mod(gparts["x"], box)
    w = box / cdim
    top = np.minimum((x / w).astype(np.int64), cdim - 1)
    tkey = (top[:, 0] * cdim + top[:, 1]) * cdim + top[:, 2]
    # position within the top cell, 21 bits per axis, interleaved (Morton)
    rel = np.clip((x - top * w) / w, 0.0, 1.0 - 1e-12)
    q = (rel * (1 << 21)).astype(np.uint64)

    def spread(v):
        v = v & np.uint64(0x1FFFFF)
        v = (v | (v << np.uint64(32))) & np.uint64(0x1F00000000FFFF)
        v = (v | (v << np.uint64(16))) & np.uint64(0x1F0000FF0000FF)
        v = (v | (v << np.uint64(8))) & np.uint64(0x100F00F00F00F00F)
        v = (v | (v << np.uint64(4))) & np.uint64(0x10C30C30C30C30C3)
        v = (v | (v << np.uint64(2))) & np.uint64(0x1249249249249249)
        return v

    mort = (spread(q[:, 0]) << np.uint64(2)) | (spread(q[:, 1]) << np.uint64(1)) | spread(q[:, 2])
    order = np.lexsort((mort, tkey))
    g = gparts[order].copy()
    tkey, mort = tkey[order], mort[order]
    cells = []

    def make(start, count, level, loc, width):
        idx = len(cells)
        cells.append([start, count, 0, [-1] * 8, loc, width])
        if count > split_size and level < max_depth:
            shift = np.uint64(3 * (20 - level))
            octant = ((mort[start:start + count] >> shift) & np.uint64(7)).astype(np.int64)
            bounds = np.searchsorted(octant, np.arange(9))  # sorted within the cell
            prog = [-1] * 8
            hw = 0.5 * width
            for k in range(8):  # octant bits: x (4), y (2), z (1)
                c0, c1 = int(bounds[k]), int(bounds[k + 1])
                if c1 > c0:
                    cl = (loc[0] + hw * ((k >> 2) & 1), loc[1] + hw * ((k >> 1) & 1),
                          loc[2] + hw * (k & 1))
                    prog[k] = make(start + c0, c1 - c0, level + 1, cl, hw)
            cells[idx][2] = 1
            cells[idx][3] = prog
        return idx

    counts = np.bincount(tkey, minlength=cdim ** 3)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    tops = []
    for t in range(cdim ** 3):
        if counts[t] > 0:
            tx, ty, tz = t // (cdim * cdim), (t // cdim) % cdim, t % cdim
            tops.append(make(int(starts[t]), int(counts[t]), 0, (tx * w, ty * w, tz * w), w))
    arr = np.zeros(len(cells), dtype=abi.GCELL_DTYPE)
    for k, (st, ct, sp, pg, loc, width) in enumerate(cells):
        arr[k] = (st, ct, sp, pg, loc, (width, width, width))
    return g, arr, np.asarray(tops, dtype=np.int32)


def top_level_pairs(tops: np.ndarray) -> np.ndarray:
    """Every unordered pair of top-level cells (the walk prunes far ones)."""
    n = len(tops)
    i, j = np.triu_indices(n, k=1)
    return np.stack([tops[i], tops[j]], axis=1).astype(np.int32)


# examples/SmallCosmoVolume/SmallCosmoVolume_hydro/small_cosmo_volume.yml:
# WMAP9 (Omega_cdm 0.2305, Omega_b 0.0455, Omega_lambda 0.724, h 0.703),
# a_begin 0.019607843 (z = 50), a 64^3 box of 142.248 Mpc (100 Mpc/h; the
# yml's softening 0.0889 Mpc = 1/25 of the 2.2226 Mpc mean separation),
# initial_temperature 7075 K. Internal units of the stand-in: length = the box,
# velocity = km/s, G = 1 (so masses are G M); H0 = 70.3 km/s/Mpc x 142.248
# Mpc = 1e4 km/s per box length.
SCV_OMEGA_CDM, SCV_OMEGA_B, SCV_OMEGA_L = 0.2305, 0.0455, 0.724
SCV_H0 = 1.0e4
SCV_A_BEGIN = 0.019607843
SCV_T_INIT = 7075.0


def small_cosmo_volume(n: int = 64, seed: int = 50, disp_rms: float = 0.2,
                       spectral_index: float = -1.5):
    """SmallCosmoVolume stand-in (BASELINE config 5): a DM-only Zel'dovich
    field turned into DM + gas pairs the way SWIFT's generate_gas_in_ics does
    (space_generate_gas, src/space.c:1747-1935).

    DM: an n^3 lattice displaced by a Gaussian random Zel'dovich field
    (displacement psi = grad of the potential of a density field with power
    P(k) ~ k^spectral_index, i.e. psi_k ~ i k delta_k / k^2, rms |psi| =
    disp_rms of the mean separation: ~0.2 at z = 50 for this box), velocity
    the linear growing mode v = a^2 H f psi (SWIFT's internal a^2 dx/dt; f = 1
    in matter domination). Each DM particle then splits (space.c:1883-1904):
    d = mean separation, the DM keeps mass (1 - Omega_b/Omega_m) and moves by
    +0.5 d Omega_b/Omega_m along the diagonal, the gas gets Omega_b/Omega_m of
    the mass and moves by -0.5 d (1 - Omega_b/Omega_m), h = d, the gas velocity
    is its gpart's. Total mass = the critical density's Omega_m share, 3 H0^2
    Omega_m / (8 pi) in G = 1 units; u = the comoving internal energy of
    7075 K gas (mu = 1.22), u_phys a^2 (SWIFT's a^(3(gamma-1)) factor).

    Returns (gas struct-part records, gpart records: the n^3 DM first, then
    the n^3 gas gparts, softening d / 25)."""
    rng = _rng(seed)
    N = n ** 3
    d = 1.0 / n
    k1 = np.fft.fftfreq(n, d=d) * 2.0 * np.pi
    kz1 = np.fft.rfftfreq(n, d=d) * 2.0 * np.pi
    kx, ky, kz = np.meshgrid(k1, k1, kz1, indexing="ij")
    k2 = kx * kx + ky * ky + kz * kz
    k2[0, 0, 0] = 1.0
    amp = np.sqrt(k2 ** (0.5 * spectral_index))
    amp[0, 0, 0] = 0.0
    noise = np.fft.rfftn(rng.standard_normal((n, n, n)))
    delta_k = noise * amp
    psi = np.empty((n, n, n, 3))
    for c, kc in enumerate((kx, ky, kz)):
        psi[..., c] = np.fft.irfftn(1j * kc * delta_k / k2, s=(n, n, n))
    psi = psi.reshape(N, 3)
    psi *= disp_rms * d / np.sqrt((psi ** 2).sum(axis=1).mean())
    g1 = (np.arange(n) + 0.5) * d
    qx, qy, qz = np.meshgrid(g1, g1, g1, indexing="ij")
    x = np.stack([qx.ravel(), qy.ravel(), qz.ravel()], axis=1) + psi
    a = SCV_A_BEGIN
    om = SCV_OMEGA_CDM + SCV_OMEGA_B
    H = SCV_H0 * np.sqrt(om / a ** 3 + SCV_OMEGA_L)
    v = a * a * H * psi
    m_tot = 3.0 * SCV_H0 ** 2 * om / (8.0 * np.pi)
    ratio = SCV_OMEGA_B / om
    m = m_tot / N
    shift_dm, shift_gas = 0.5 * d * ratio, 0.5 * d * (1.0 - ratio)
    eps = d / 25.0
    gp = abi.new_gparts(2 * N)
    gp["id_or_neg_offset"][:N] = 2 * np.arange(1, N + 1)
    gp["id_or_neg_offset"][N:] = -np.arange(N)  # linked to gas part j (space.c:1880)
    gp["x"][:N] = np.mod(x + shift_dm, 1.0)
    gp["x"][N:] = np.mod(x - shift_gas, 1.0)
    gp["v_full"][:N] = v
    gp["v_full"][N:] = v
    gp["mass"][:N] = m * (1.0 - ratio)
    gp["mass"][N:] = m * ratio
    gp["epsilon"] = eps
    gp["time_bin"] = 1
    gp["type"][:N] = 1
    gp["type"][N:] = 0
    gas = abi.new_parts(N)
    gas["id"] = 2 * np.arange(1, N + 1) + 1
    gas["x"] = gp["x"][N:]
    gas["v"] = v.astype(np.float32)
    gas["mass"] = m * ratio
    gas["h"] = d
    k_B, m_p, mu = 1.380649e-16, 1.67262192e-24, 1.22
    u_phys = SCV_T_INIT * k_B / (mu * m_p * (GAMMA - 1.0)) / 1e10  # (km/s)^2
    gas["u"] = u_phys * a * a
    gas["time_bin"] = 1
    gas["visc_alpha"] = 0.1
    return gas, gp
