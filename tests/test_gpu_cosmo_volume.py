"""BASELINE config 5 at its size: the SmallCosmoVolume stand-in's first step
(bench.py --workload cosmo), 64^3 gas + 64^3 DM, against the fp64 oracle.

  * ics.small_cosmo_volume(64): a Zel'dovich DM field split into DM + gas
    pairs as space_generate_gas does (src/space.c:1747-1935);
  * hydro: the whole SPHENIX chain (density, ghost from h = the mean
    separation, gradient, extra ghost, force, end force) with the WMAP9
    cosmology of small_cosmo_volume.yml at a = 0.0198 (a, H, a^2 H, the
    scale-factor powers, dt_alpha of time bin 47) vs the oracle chain:
    exact counts, h, every chain field at check_chain's tolerances;
  * gravity: the cell tree (8^3 top cells split to <= 50 gparts, 37k cells),
    the recursive walk (P2P, M2P, M2L, L2L, L2P; r_cut_max 4.5 r_s) + the PM
    mesh (64^3, a_smooth 1.25) vs the oracle's grav_tree and pm_mesh, first
    with the geometric MAC (theta_cr 0.7), then with the yml's adaptive MAC
    (epsilon_fmm 0.001, multipole_accept.h:81-170) fed the same
    old_a_grav_norm = |a_tree + a_mesh / G| (gravity.h:244-253): identical
    P2P / M2P / M2L counts, a_grav and potential to 2e-5 of |a|, the mesh
    fields to 2e-6 of their maximum.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
from test_gpu_physics import check_chain, gpu_chain, oracle_chain
from swift_subtask_dev_amd import abi, cosmo, ics

pytestmark = pytest.mark.gpu

N_MESH = 64
R_S = 1.25 / N_MESH


def grav_params(adaptive):
    G = abi.GravParams(1, (C.c_float * 3)(1, 1, 1), 1.0 / R_S, 0.1 * R_S, abi.NUM_TIME_BINS)
    G.theta_crit = 0.7
    G.adaptive_tolerance = 1e-3
    G.use_advanced_MAC = 1 if adaptive else 0
    G.r_cut_max = 4.5 * R_S
    return G


@pytest.fixture(scope="module")
def volume():
    gas, gp = ics.small_cosmo_volume(64)
    _, P = cosmo.small_cosmo_volume_params()
    gas["time_bin"] = cosmo.SCV_FIRST_BIN
    return gas, gp, P


def test_small_cosmo_volume_hydro_chain_vs_f64(gpu_ctx, volume):
    gas, _, P = volume
    assert abs(P.a - 0.01976) < 1e-4 and P.H > 1e6
    g, rg = gpu_chain(gpu_ctx, gas, P)
    o, ro = oracle_chain(gas, P)
    print(f"\nhydro: gpu {rg} oracle {ro}")
    check_chain(g, rg, o, ro, np.ones(len(gas), dtype=bool))
    # the expansion term is live: a^2 H r^2 dominates dv.dx at z = 50
    assert np.abs(o["div_v"]).max() > 0


def _gpu_gravity(ctx, g, cells, tops, pairs, G):
    from swift_subtask_dev_amd import lib
    gs = lib.GravSpace(ctx)
    gs.upload(g)
    gs.set_tree(cells)
    st = gs.tree(G, tops, pairs)
    gs.pm_mesh(N_MESH, 1.0, R_S, 1.0)
    out = abi.copy_parts(g)
    gs.download(out)
    gs.close()
    return out, st


def _oracle_gravity(g, cells, tops, pairs, G):
    o = abi.copy_parts(g)
    st = np.zeros(6, dtype=np.int64)
    O.fn("f64", "grav_tree")(o.ctypes.data, len(o), cells.ctypes.data, len(cells),
                             tops.ctypes.data, len(tops), pairs.ctypes.data, len(pairs),
                             C.byref(G), st.ctypes.data, None)
    pot = np.zeros((N_MESH,) * 3)
    O.fn("f64", "pm_mesh")(o.ctypes.data, len(o), N_MESH, 1.0, R_S, 1.0, pot.ctypes.data)
    return o, st


def _compare_gravity(gg, go, st_g, st_o):
    assert [st_g["n_pp"], st_g["n_m2p"], st_g["n_m2l"], st_g["n_pp_tasks"],
            st_g["n_skipped"], st_g["n_pp_truncated"]] == list(st_o), (st_g, st_o)
    a_o = go["a_grav"].astype(np.float64)
    scale = np.linalg.norm(a_o, axis=1)
    e = np.linalg.norm(gg["a_grav"].astype(np.float64) - a_o, axis=1) / np.maximum(scale, 1e-30)
    assert e.max() < 2e-5, (e.max(), int(np.argmax(e)))
    ep = np.abs(gg["potential"] - go["potential"]) / np.maximum(np.abs(go["potential"]), 1e-30)
    assert ep.max() < 2e-5, ep.max()
    for f in ("a_grav_mesh", "potential_mesh"):
        a, b = gg[f].astype(np.float64), go[f].astype(np.float64)
        assert np.abs(a - b).max() <= 2e-6 * np.abs(b).max(), f


def test_small_cosmo_volume_gravity_vs_f64(gpu_ctx, volume):
    _, gp, _ = volume
    g, cells, tops = ics.gravity_tree(gp, 8, split_size=50)
    pairs = ics.top_level_pairs(tops)
    assert len(g) == 2 * 64 ** 3 and len(cells) > 30000
    G = grav_params(adaptive=False)
    gg, st_g = _gpu_gravity(gpu_ctx, g, cells, tops, pairs, G)
    go, st_o = _oracle_gravity(g, cells, tops, pairs, G)
    print(f"\ngeometric MAC: gpu {st_g} oracle {list(st_o)}")
    _compare_gravity(gg, go, st_g, st_o)
    assert st_g["n_m2l"] > 0
    # the adaptive MAC on the |a| the oracle's geometric step recorded
    g["old_a_grav_norm"] = np.linalg.norm(go["a_grav"].astype(np.float64)
                                          + go["a_grav_mesh"].astype(np.float64), axis=1)
    G = grav_params(adaptive=True)
    gg, st_g = _gpu_gravity(gpu_ctx, g, cells, tops, pairs, G)
    go, st_o = _oracle_gravity(g, cells, tops, pairs, G)
    print(f"adaptive MAC: gpu {st_g} oracle {list(st_o)}")
    _compare_gravity(gg, go, st_g, st_o)
