"""Build libswifthip (gfx950) and the SWIFT-signature adapter in-tree.

Run as `python -m swift_subtask_dev_amd.build` or via __graft_entry__.build().
hipcc cross-compiles for gfx950 without a GPU; the .so files are written next
to this file so they travel to the GPU box with the repo snapshot.

The SPH kernel is a build-time choice, as SWIFT's configure --with-kernel
(configure.ac:2107-2137): libswifthip.so / libswifthip_swift.so use the cubic
spline (SWIFT's default), libswifthip_wc2.so / libswifthip_swift_wc2.so the
Wendland C2 kernel (kernel_hydro.h:121-147), built with
-DSWH_KERNEL_WENDLAND_C2. Both export the same C ABI.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = REPO / "include"
LIB = PKG / "libswifthip.so"
ADAPTER = PKG / "libswifthip_swift.so"

# kernel -> (library, adapter, object dir, defines)
VARIANTS = {
    "cubic-spline": (LIB, ADAPTER, "_obj", []),
    "wendland-c2": (PKG / "libswifthip_wc2.so", PKG / "libswifthip_swift_wc2.so", "_obj_wc2",
                    ["-DSWH_KERNEL_WENDLAND_C2"]),
}

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


def build_variant(kernel: str, force: bool = False, verbose: bool = False,
                  jobs: int = 4) -> Path:
    lib, adapter, objname, defines = VARIANTS[kernel]
    objdir = PKG / objname
    objdir.mkdir(exist_ok=True)
    headers = [CSRC / h for h in HIP_HEADERS] + [INCLUDE / "swifthip.h", INCLUDE / "swift_compat.h"]
    common = [
        "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
        "-Wno-unused-function", "-Wno-unused-variable",
        f"-I{INCLUDE}", f"-I{CSRC}", "-fvisibility=hidden",
        "-DSWH_BUILD", *defines,
        # experiment flags (e.g. -DSWH_M2P_PROF); any set forces a full rebuild
        *os.environ.get("SWH_EXTRA_FLAGS", "").split(),
    ]
    # the flags of the objects in objdir: a build with other flags (an
    # experiment's SWH_EXTRA_FLAGS, or a plain build after one) rebuilds all
    stamp = objdir / "flags.stamp"
    flags = " ".join(common)
    if not stamp.exists() or stamp.read_text() != flags:
        force = True
    objs, cmds = [], []
    for src in HIP_SOURCES:
        s = CSRC / src
        o = objdir / (src + ".o")
        objs.append(o)
        if force or _stale(o, [s] + headers):
            cmds.append([_hipcc(), *common, "-c", str(s), "-o", str(o)])
    for c in cmds:
        if verbose:
            print(" ".join(c))
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, cmds))
    if force or _stale(lib, objs):
        _run([_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-Wl,-Bsymbolic",
              "-o", str(lib), *map(str, objs), "-lhipfft"])
    # SWIFT-signature adapter: plain C against the SWIFT field-name mirrors.
    asrc = CSRC / "swh_swift_adapter.c"
    if asrc.exists() and (force or _stale(adapter, [asrc, lib, INCLUDE / "swifthip.h",
                                                   INCLUDE / "swift_compat.h",
                                                   INCLUDE / "swifthip_swift.h"])):
        _run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-shared", "-Wall", f"-I{INCLUDE}", *defines,
              "-o", str(adapter), str(asrc), f"-L{PKG}", f"-l:{lib.name}",
              "-Wl,-rpath,$ORIGIN"])
    stamp.write_text(flags)
    return lib


def build(force: bool = False, verbose: bool = False) -> Path:
    for kernel in VARIANTS:
        build_variant(kernel, force=force, verbose=verbose)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose="-v" in sys.argv)
    print(f"built {', '.join(str(v[0].name) for v in VARIANTS.values())}")
