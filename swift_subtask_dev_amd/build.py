"""Build libswifthip.so (gfx950) and the SWIFT-signature adapter in-tree.

Run as `python -m swift_subtask_dev_amd.build` or via __graft_entry__.build().
hipcc cross-compiles for gfx950 without a GPU; the .so files are written next
to this file so they travel to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = REPO / "include"
LIB = PKG / "libswifthip.so"
ADAPTER = PKG / "libswifthip_swift.so"

HIP_SOURCES = ["swh_api.hip", "swh_tasks.hip", "swh_space.hip", "swh_hydro.hip", "swh_grav.hip",
               "swh_mesh.hip"]
HIP_HEADERS = ["swh_internal.h", "swh_physics.h", "swh_space.h", "swh_gather.h", "swh_wave.h",
               "swh_list.h", "swh_mpole.h"]


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    return str(Path(rocm) / "bin" / "hipcc")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {' '.join(cmd[:3])} ...")


def build(force: bool = False, verbose: bool = False) -> Path:
    objdir = PKG / "_obj"
    objdir.mkdir(exist_ok=True)
    headers = [CSRC / h for h in HIP_HEADERS] + [INCLUDE / "swifthip.h", INCLUDE / "swift_compat.h"]
    objs = []
    common = [
        "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
        "-Wno-unused-function", "-Wno-unused-variable",
        f"-I{INCLUDE}", f"-I{CSRC}", "-fvisibility=hidden",
        "-DSWH_BUILD",
    ]
    for src in HIP_SOURCES:
        s = CSRC / src
        o = objdir / (src + ".o")
        objs.append(o)
        if force or _stale(o, [s] + headers):
            cmd = [_hipcc(), *common, "-c", str(s), "-o", str(o)]
            if verbose:
                print(" ".join(cmd))
            _run(cmd)
    if force or _stale(LIB, objs):
        _run([_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs),
              "-lhipfft"])
    # SWIFT-signature adapter: plain C against the SWIFT field-name mirrors.
    asrc = CSRC / "swh_swift_adapter.c"
    if asrc.exists() and (force or _stale(ADAPTER, [asrc, LIB, INCLUDE / "swifthip.h",
                                                   INCLUDE / "swift_compat.h",
                                                   INCLUDE / "swifthip_swift.h"])):
        _run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-shared", "-Wall", f"-I{INCLUDE}",
              "-o", str(ADAPTER), str(asrc), f"-L{PKG}", "-lswifthip",
              f"-Wl,-rpath,$ORIGIN"])
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose="-v" in sys.argv)
    print(f"built {LIB}")
