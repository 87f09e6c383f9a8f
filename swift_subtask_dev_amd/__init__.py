"""swift_subtask_dev_amd — MI355X (gfx950) HIP implementation of SWIFT's SPH
density/gradient/force neighbour loops and P2P gravity, behind SWIFT's own
per-task entry points (include/swifthip_swift.h) and a batch C ABI
(include/swifthip.h).

Python is host plumbing only: the compute path is libswifthip.so (HIP);
``swift_subtask_dev_amd.lib`` fails loudly when the library has not been built.
"""
from . import abi, ics  # noqa: F401

__all__ = ["abi", "ics", "lib"]
