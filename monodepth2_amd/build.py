"""In-tree build of the HIP library (libmd2hot.so) for gfx950.

`python -m monodepth2_amd.build` or `__graft_entry__.build()`.  The .so lands
next to its source (monodepth2_amd/csrc/) so it travels to the GPU box with the
repository snapshot; it is git-ignored.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB_NAME = "libmd2hot.so"
LIB_PATH = os.path.join(CSRC, LIB_NAME)
SOURCES = ["md2hot.hip", "decoder.hip", "pose.hip", "augment.hip", "bnorm.hip", "pool.hip"]
ARCH = os.environ.get("MD2_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libmd2hot.so)")


def needs_build() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(INCLUDE, "md2hot.h"),
                                                       os.path.join(CSRC, "md2_bf16.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB_PATH
    tmp = LIB_PATH + ".tmp"
    cmd = [hipcc(), "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared",
           "-I" + INCLUDE, "-o", tmp] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
