"""Per-rank halo volume of bench.py's block decompositions (decomp.HaloPlan),
computed on the CPU from the bench's own inputs: owned and halo particles per
rank, peers, and the bytes one halo refresh moves (32-byte records,
SWH_HALO_RECORD_FLOATS = 8) for the Sedov 128^3 headline box and the config-5
gas at 1/2/4/8 ranks. The halo reach is the bench's 1.01 gamma h_max; h is
the input's (Sedov: eta / n, which the ghost keeps to within a few per cent
on the lattice; config 5: the ICs' h) -- a plan estimate, not a converged run.

usage: python tools/halo_volume.py [out.json]
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from swift_subtask_dev_amd import abi, decomp, ics  # noqa: E402

GAMMA = 1.825742
LINK_GBPS = 153e9  # one xGMI link per direction (MI355X_MICROARCH.md)


def plan_stats(x, h, box, world):
    reach = 1.01 * GAMMA * float(h.max())
    ranks = []
    for r in range(world):
        p = decomp.HaloPlan(x, box, world, r, reach)
        sent = sum(len(v) for v in p.send.values())
        recv = sum(c for _, c in p.recv.values())
        per_peer = max([len(v) for v in p.send.values()] + [0])
        ranks.append({"rank": r, "owned": int(p.n_owned), "halo": int(len(p.halo)),
                      "peers": len(p.peers()), "records_sent": int(sent),
                      "records_received": int(recv),
                      "bytes_sent": int(sent * abi.HALO_RECORD_FLOATS * 4),
                      "largest_peer_bytes": int(per_peer * abi.HALO_RECORD_FLOATS * 4)})
    worst = max(ranks, key=lambda q: q["bytes_sent"])
    return {"world": world, "dims": list(decomp.block_dims(world)), "reach": reach,
            "ranks": ranks,
            "halo_over_owned_max": max(q["halo"] / max(1, q["owned"]) for q in ranks),
            "bytes_sent_max": worst["bytes_sent"],
            # every peer on its own xGMI link (a fully connected 8-GPU node):
            # the refresh is bound by the largest single transfer
            "link_time_us_model": max(q["largest_peer_bytes"] for q in ranks) / LINK_GBPS * 1e6}


def main():
    out = {"note": __doc__.strip().splitlines()[0] + " (see the module docstring)",
           "record_bytes": abi.HALO_RECORD_FLOATS * 4, "xgmi_link_bytes_per_s": LINK_GBPS}
    sed = ics.sedov_slabs(128, 1)
    out["sedov128"] = [plan_stats(sed["x"], sed["h"], (1.0, 1.0, 1.0), w) for w in (2, 4, 8)]
    del sed
    gas, _ = ics.small_cosmo_volume(64)
    out["cosmo64"] = [plan_stats(gas["x"], gas["h"], (1.0, 1.0, 1.0), w) for w in (2, 4, 8)]
    text = json.dumps(out, indent=1)
    if len(sys.argv) > 1:
        Path(sys.argv[1]).write_text(text + "\n")
    for k in ("sedov128", "cosmo64"):
        for s in out[k]:
            print(f"{k} world {s['world']}: halo/owned <= {s['halo_over_owned_max']:.3f}, "
                  f"max bytes sent {s['bytes_sent_max'] / 1e6:.2f} MB, "
                  f"largest transfer at one link {s['link_time_us_model']:.1f} us")


if __name__ == "__main__":
    main()
