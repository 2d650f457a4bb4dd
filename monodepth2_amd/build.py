"""In-tree build of the HIP library (libmd2hot.so) for gfx950.

`python -m monodepth2_amd.build` or `__graft_entry__.build()`.  The .so lands
next to its source (monodepth2_amd/csrc/) so it travels to the GPU box with the
repository snapshot; it is git-ignored.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB_NAME = "libmd2hot.so"
LIB_PATH = os.path.join(CSRC, LIB_NAME)
SOURCES = ["md2hot.hip", "decoder.hip", "pose.hip", "augment.hip", "bnorm.hip", "pool.hip", "adam.hip", "disphead.hip", "stem.hip", "bias_act.hip", "conv.hip", "direct.hip", "glue.hip"]
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
    if any(os.path.getmtime(d) > t for d in deps):
        return True
    # per-source flags changed (they are part of the build id, not of any mtime).  The
    # id is read from the file's bytes, NOT by loading the library: a dlopen here would
    # pin this copy in the process, and after a rebuild os.replace()s the file a later
    # _lib.lib() would get the stale mapping back from dlopen's cache
    return built_id(LIB_PATH) != source_hash()


def built_id(path: str):
    """The MD2_BUILD_ID baked into a built library (glue.hip stores it behind a marker
    string), read from the file without loading it; None if absent."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(BUILD_ID_MARKER)
    if i < 0:
        return None
    i += len(BUILD_ID_MARKER)
    return data[i:i + 16].decode("ascii", errors="replace")


BUILD_ID_MARKER = b"md2-build-id:"


# Per-source extra flags.  md2hot.hip: no SLP vectorisation — packed-f32 VALU
# (v_pk_fma_f32 / v_pk_mul_f32) issues no faster than two scalar ops on gfx950 and the
# register pairs it needs cost ~100 v_mov per row step of the photometric kernels;
# measured: photo_bwd 0.306 -> 0.287 ms at B=12 640x192.
# disphead.hip: also no SLP — the vectorised weight-gradient accumulation became
# v_pk_fma_f32 whose src1 op_sel has the low lane read the pair's high dword, and those
# instructions (taps 1 and 7, and only they) gave intermittently different low-lane
# results when another process shared the GPU; tests/test_isa_guard.py
# keeps that encoding out of the whole library (glue.hip's input normalisation had it
# too, on an SGPR pair: no SLP there either).
# md2hot.hip also with LLVM's iterative ILP scheduler: forward 0.1259 -> 0.1240, backward
# 0.2426 -> 0.2387 ms (means of three alternated tools/hot_bench.py runs; max-ilp,
# max-memory-clause, iterative-minreg and iterative-maxocc measured slower or equal).
# conv.hip (the x6 GEMMs) with LLVM's max-ILP scheduler: captured step 11.65 -> 11.54 ms
# (three alternated runs each, pinned convolution choices; iterative-ilp equal to the
# default there); bnorm.hip + decoder.hip with it too: 11.721 -> 11.693 ms (three
# alternated pairs, every pair faster); stem.hip and direct.hip were slower with it.
FLAGS = {"md2hot.hip": ["-fno-slp-vectorize", "-mllvm", "--amdgpu-sched-strategy=iterative-ilp"],
         "conv.hip": ["-mllvm", "--amdgpu-sched-strategy=max-ilp"],
         "bnorm.hip": ["-mllvm", "--amdgpu-sched-strategy=max-ilp"],
         "decoder.hip": ["-mllvm", "--amdgpu-sched-strategy=max-ilp"],
         "disphead.hip": ["-fno-slp-vectorize"], "glue.hip": ["-fno-slp-vectorize"]}


def source_hash() -> str:
    """Hash of everything the library is built from (sources, headers, per-source
    flags, target architecture): baked into the library as md2_build_id() and checked
    against the tree by _lib.lib(), so a stale prebuilt .so cannot load silently."""
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(INCLUDE, "md2hot.h"),
                                                          os.path.join(CSRC, "md2_bf16.h")]:
        h.update(os.path.basename(path).encode())
        with open(path, "rb") as f:
            h.update(f.read())
    h.update(repr(sorted(FLAGS.items())).encode())
    h.update(ARCH.encode())
    return h.hexdigest()[:16]


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB_PATH
    import concurrent.futures as cf
    objdir = os.path.join(CSRC, "obj")
    os.makedirs(objdir, exist_ok=True)
    base = [hipcc(), "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-I" + INCLUDE]
    bid = ['-DMD2_BUILD_ID="%s"' % source_hash()]

    def compile_one(src):
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        cmd = base + FLAGS.get(src, []) + (bid if src == "glue.hip" else []) + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB_PATH + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
