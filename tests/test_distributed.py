"""Multi-process decomposition (bench.py's weak-scaling layout) on CPU with
the gloo backend, world_size 2 and 3: every rank holds its x-slab + a
read-only halo (swift_subtask_dev_amd/decomp.py) and evaluates the loops of
its own particles; the union over ranks must equal the single-domain result
and the interaction counts must add up, with no data-path collective (only
the test's final gather). The oracle stands in for the GPU here (no GPU in
CI); the GPU path runs the same decomposition in bench.py."""
from __future__ import annotations

import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, queue):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "tests"))
    import oracle_lib as O
    from swift_subtask_dev_amd import abi, decomp, ics

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    parts = ics.sedov_slabs(n, world, pert=0.2, seed=42)
    box = (float(world), 1.0, 1.0)
    P = abi.default_hydro_params(box, True)
    P.max_active_bin = 1
    hmax = float(parts["h"].max()) * 1.825742
    local, n_owned = decomp.slab_local_set(parts, rank, world, box[0], 1.02 * hmax)
    O.fn("f32", "init_parts")(local.ctypes.data, len(local), C.byref(P))
    nd = O.fn("f64", "box_density")(local.ctypes.data, len(local), C.byref(P), None)
    owned = local[:n_owned]
    res = {"id": owned["id"].copy(), "rho": owned["rho"].copy(),
           "div_v": owned["div_v"].copy(), "n": nd}
    out = [None] * world
    dist.all_gather_object(out, res)
    if rank == 0:
        queue.put(out)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_slab_decomposition_matches_single_domain(world):
    from swift_subtask_dev_amd import abi, ics
    import oracle_lib as O

    n = 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    parts = ics.sedov_slabs(n, world, pert=0.2, seed=42)
    P = abi.default_hydro_params((float(world), 1.0, 1.0), True)
    P.max_active_bin = 1
    O.fn("f32", "init_parts")(parts.ctypes.data, len(parts), C.byref(P))
    n_all = O.fn("f64", "box_density")(parts.ctypes.data, len(parts), C.byref(P), None)
    assert sum(r["n"] for r in out) == n_all
    ids = np.concatenate([r["id"] for r in out])
    assert len(ids) == len(parts) and len(np.unique(ids)) == len(parts)
    rho = np.concatenate([r["rho"] for r in out])
    order = np.argsort(ids)
    ref = parts[np.argsort(parts["id"])]
    assert np.array_equal(rho[order], ref["rho"])
    assert np.array_equal(np.concatenate([r["div_v"] for r in out])[order], ref["div_v"])
