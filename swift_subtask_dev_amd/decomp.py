"""Multi-GPU decomposition of the hot path.

The periodic box is split into a grid of blocks, one per rank (one process per
GPU): 2 = 2x1x1, 4 = 2x2x1, 8 = 2x2x2 (slabs would be too thin at 8 GPUs).
A rank owns the particles of its block and holds a read-only halo: every
particle whose distance to the block is below the interaction reach
(gamma h_max: no pair with r < max(H_i, H_j) can reach further). The loops
then need nothing from other ranks while they run: SPH gathers have no
cross-cell reduction (every directed pair is evaluated by the owner of i).
Between loop phases the fields the next phase reads from neighbours are
refreshed point-to-point (SURVEY 8e "Collective / exchange"):

  after the ghost        h, rho, pressure, soundspeed, f, balsara
  after the extra ghost  alpha_visc, alpha_diff

Halo particles keep their real time bins (the limiter reads them); ownership
is separate: libswifthip's swh_space_set_owned marks every upload index past
the owned block as foreign (SWIFT's foreign cells), and the CPU oracle, which
has no such notion, gets halo_time_bin copies instead (tests only).

The exchange plan is a pure function of the global particle set, so every
rank derives the same plan with no communication: a rank's local array is its
owned particles (ascending global index) followed by its halo grouped by
owning rank (ascending global index within each group); what rank r sends to
rank q is exactly q's halo group from r, in the same order.
"""
from __future__ import annotations

import numpy as np

from . import abi

# halo record: the fields the next loop phase reads from neighbours
HALO_FIELDS = ("h", "rho", "pressure", "soundspeed", "f", "balsara", "visc_alpha", "diff_alpha")
HALO_AFTER_GHOST = abi.HALO_H | abi.HALO_RHO | abi.HALO_PC | abi.HALO_F_BALSARA
HALO_AFTER_EXTRA_GHOST = abi.HALO_ALPHAS


def block_dims(world: int):
    """Blocks per dimension: 1 -> 1x1x1, 2 -> 2x1x1, 4 -> 2x2x1, 8 -> 2x2x2;
    other counts split the currently longest dimension by the smallest prime
    factor left."""
    dims = [1, 1, 1]
    left = world
    while left > 1:
        p = next(f for f in range(2, left + 1) if left % f == 0)
        k = dims.index(min(dims))
        dims[k] *= p
        left //= p
    return tuple(dims)


def block_of(x: np.ndarray, box, dims) -> np.ndarray:
    """Owning rank of each position (rank = (bx * ny + by) * nz + bz)."""
    b = []
    for k in range(3):
        xs = np.mod(x[:, k], box[k])
        b.append(np.minimum((xs / box[k] * dims[k]).astype(np.int64), dims[k] - 1))
    return (b[0] * dims[1] + b[1]) * dims[2] + b[2]


def block_bounds(rank: int, box, dims):
    bz = rank % dims[2]
    by = (rank // dims[2]) % dims[1]
    bx = rank // (dims[1] * dims[2])
    lo = np.array([bx * box[0] / dims[0], by * box[1] / dims[1], bz * box[2] / dims[2]])
    hi = np.array([(bx + 1) * box[0] / dims[0], (by + 1) * box[1] / dims[1],
                   (bz + 1) * box[2] / dims[2]])
    return lo, hi


def distance_to_block(x: np.ndarray, lo, hi, box) -> np.ndarray:
    """Periodic Euclidean distance of each position to the box [lo, hi)."""
    d2 = np.zeros(len(x))
    for k in range(3):
        L = box[k]
        xs = np.mod(x[:, k], L)
        inside = (xs >= lo[k]) & (xs < hi[k])
        below = np.mod(lo[k] - xs, L)  # distance up to the block's lower face
        above = np.mod(xs - hi[k], L)  # distance past its upper face
        dk = np.where(inside, 0.0, np.minimum(below, above))
        if hi[k] - lo[k] >= L:  # the block spans the whole dimension
            dk[:] = 0.0
        d2 += dk * dk
    return np.sqrt(d2)


class HaloPlan:
    """One rank's view of the decomposition (see module docstring)."""

    def __init__(self, x: np.ndarray, box, world: int, rank: int, reach: float):
        self.world, self.rank = world, rank
        self.dims = block_dims(world)
        self.box = tuple(float(b) for b in box)
        owner = block_of(x, self.box, self.dims)
        self.owned = np.nonzero(owner == rank)[0]
        self.n_owned = len(self.owned)
        # halo[q] for every rank q: foreign particles within reach of q's block
        halos = []
        for q in range(world):
            lo, hi = block_bounds(q, self.box, self.dims)
            near = distance_to_block(x, lo, hi, self.box) < reach
            halos.append(np.nonzero(near & (owner != q))[0])
        mine = halos[rank]
        self.recv = {}  # source rank -> (first local index, count)
        groups = []
        start = self.n_owned
        for src in range(world):
            if src == rank:
                continue
            g = mine[owner[mine] == src]
            if len(g):
                self.recv[src] = (start, len(g))
                groups.append(g)
                start += len(g)
        self.halo = np.concatenate(groups) if groups else np.zeros(0, dtype=np.int64)
        self.n_local = self.n_owned + len(self.halo)
        self.send = {}  # destination rank -> local indices of owned particles, q's order
        for dst in range(world):
            if dst == rank:
                continue
            g = halos[dst][owner[halos[dst]] == rank]
            if len(g):
                self.send[dst] = np.searchsorted(self.owned, g).astype(np.int32)
        self.recv_idx = {src: np.arange(s, s + c, dtype=np.int32)
                         for src, (s, c) in self.recv.items()}

    def local_set(self, parts: np.ndarray, halo_time_bin=None) -> np.ndarray:
        """Owned particles, then the halo groups. halo_time_bin: overwrite the
        halo's time bins (only for the CPU oracle, which has no ownership)."""
        out = abi.new_parts(self.n_local)
        out[: self.n_owned] = parts[self.owned]
        out[self.n_owned:] = parts[self.halo]
        if halo_time_bin is not None:
            out["time_bin"][self.n_owned:] = halo_time_bin
        return out

    def peers(self):
        return sorted(set(self.send) | set(self.recv))


def exchange(plan: HaloPlan, dist, pack, unpack, alloc):
    """One halo refresh: for every peer, pack what it needs from us, swap
    buffers point-to-point (one batched group of isend/irecv, no collective),
    unpack what we received. pack(dst, buf) fills buf with the records of
    plan.send[dst]; unpack(src, buf) applies buf to plan.recv_idx[src];
    alloc(n) returns a send/receive buffer of n halo records."""
    ops, recvs = [], []
    for q in plan.peers():
        if q in plan.send:
            sbuf = alloc(len(plan.send[q]))
            pack(q, sbuf)
            ops.append(dist.P2POp(dist.isend, sbuf, q))
        if q in plan.recv:
            rbuf = alloc(plan.recv[q][1])
            ops.append(dist.P2POp(dist.irecv, rbuf, q))
            recvs.append((q, rbuf))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for q, rbuf in recvs:
        unpack(q, rbuf)


class DeviceHalo:
    """Halo refresh of a libswifthip swh_space between loop phases: pack on
    the space's stream, swap point-to-point (exchange), unpack on the same
    stream. With RCCL ("nccl") the buffers stay in HBM: the collective stream
    waits on ours before sending and ours waits on it before unpacking. With
    gloo (tests: several ranks on one GPU) they are staged through the host.
    The space is bound to `stream`; every buffer is allocated on it, so the
    caching allocator never hands one back before the stream has used it."""

    RECORD_FLOATS = 8  # SWH_HALO_RECORD_FLOATS

    def __init__(self, plan: HaloPlan, sp, dist, torch, stream):
        self.plan, self.sp, self.dist, self.torch, self.stream = plan, sp, dist, torch, stream
        self.host = dist.get_backend() == "gloo"
        self.dev = torch.device("cuda", torch.cuda.current_device())
        sp.set_stream(stream.cuda_stream)
        with torch.cuda.stream(stream):
            self.send_idx = {q: torch.from_numpy(v).to(self.dev) for q, v in plan.send.items()}
            self.recv_idx = {q: torch.from_numpy(v).to(self.dev)
                             for q, v in plan.recv_idx.items()}

    def refresh(self, fields: int) -> None:
        torch, sp, nrec = self.torch, self.sp, self.RECORD_FLOATS

        def alloc(n):
            return torch.empty(n * nrec, dtype=torch.float32,
                               device="cpu" if self.host else self.dev)

        def pack(q, buf):
            idx = self.send_idx[q]
            dbuf = torch.empty(len(idx) * nrec, dtype=torch.float32,
                               device=self.dev) if self.host else buf
            sp.pack_halo(idx.data_ptr(), len(idx), dbuf.data_ptr())
            if self.host:
                buf.copy_(dbuf)  # synchronous on the bound stream

        def unpack(q, buf):
            idx = self.recv_idx[q]
            dbuf = buf.to(self.dev) if self.host else buf
            sp.unpack_halo(idx.data_ptr(), len(idx), dbuf.data_ptr(), fields)

        with torch.cuda.stream(self.stream):
            exchange(self.plan, self.dist, pack, unpack, alloc)


def pack_host(parts: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """Halo records of parts[idx] on the host (the CPU oracle's side)."""
    rec = np.empty((len(idx), len(HALO_FIELDS)), dtype=np.float32)
    for k, f in enumerate(HALO_FIELDS):
        rec[:, k] = parts[f][idx]
    return rec


def unpack_host(parts: np.ndarray, idx: np.ndarray, rec: np.ndarray, fields: int) -> None:
    groups = [(abi.HALO_H, ("h",)), (abi.HALO_RHO, ("rho",)),
              (abi.HALO_PC, ("pressure", "soundspeed")), (abi.HALO_F_BALSARA, ("f", "balsara")),
              (abi.HALO_ALPHAS, ("visc_alpha", "diff_alpha"))]
    for bit, names in groups:
        if fields & bit:
            for f in names:
                parts[f][idx] = rec[:, HALO_FIELDS.index(f)]


def slab_local_set(parts: np.ndarray, rank: int, world: int, box_x: float, reach: float,
                   halo_time_bin: int = 2):
    """Owned + halo particles of `rank`'s x-slab of a periodic box of length
    box_x (the weak-scaling layout of bench.py --scaling weak). Returns (local
    AoS array, n_owned): owned particles first, then the halo with
    time_bin = halo_time_bin (CPU oracle use; the GPU path uses set_owned)."""
    lo, hi = rank * box_x / world, (rank + 1) * box_x / world
    x = np.mod(parts["x"][:, 0], box_x)
    owned = (x >= lo) & (x < hi)
    if world == 1:
        return abi.copy_parts(parts), len(parts)
    d_lo = np.mod(lo - x, box_x)
    d_hi = np.mod(x - hi, box_x)
    halo = (~owned) & ((d_lo <= reach) | (d_hi < reach))
    own_idx = np.nonzero(owned)[0]
    halo_idx = np.nonzero(halo)[0]
    out = abi.new_parts(len(own_idx) + len(halo_idx))
    out[: len(own_idx)] = parts[own_idx]
    out[len(own_idx):] = parts[halo_idx]
    if halo_time_bin is not None:
        out["time_bin"][len(own_idx):] = halo_time_bin
    return out, len(own_idx)


def gravity_owned_cells(cells: np.ndarray, tops, rank: int, world: int, box) -> np.ndarray:
    """Tree-gravity ownership of one rank (swh_gspace_set_owned_cells): a top
    cell belongs to the rank whose block holds its centre (the same block grid
    as the hydro decomposition), and every cell to its top cell's owner
    (whole subtrees). gparts and multipoles stay replicated on every rank
    (i-cells owned, j-cells read-only), so no data moves while the
    walk, P2P, M2P, M2L and the down pass run."""
    dims = block_dims(world)
    tops = np.asarray(tops, dtype=np.int64)
    centre = np.asarray(cells["loc"][tops], dtype=np.float64) + 0.5 * np.asarray(
        cells["width"][tops], dtype=np.float64)
    own_top = block_of(centre, box, dims) == rank
    owned = np.zeros(len(cells), dtype=np.uint8)
    stack = [int(t) for t, o in zip(tops, own_top) if o]
    while stack:
        c = stack.pop()
        owned[c] = 1
        if cells["split"][c]:
            stack.extend(int(p) for p in cells["progeny"][c] if p >= 0)
    return owned
