"""Launch-duplication probes (DESIGN.md §8 / §9 "what the step's launches cost"): build a
variant of libmd2hot.so in which every launch of one kind is issued twice — the kinds
below are idempotent (they rewrite the same outputs from unchanged inputs), so the
results stay right and the step's extra time is that kind's marginal cost inside the
captured two-stream step, overlap included.

    python tools/dup_probe.py KIND [KIND ...]      # builds abx/dup_<KIND>/libmd2hot.so
    MD2_LIB=abx/dup_<KIND>/libmd2hot.so python bench.py --pmc 0 --no-cpu-baseline ...

Alternate the variant with the in-tree library on one box (the step spreads ~7 % box to
box).  A probe that changes the numerics (e.g. skipping a pass) is no probe: the
photometric kernels' cost depends on where the warped samples land.
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "monodepth2_amd", "csrc")

# kind -> (source, regex of the launch statement to repeat)
KINDS = {
    "bn_stats": ("bnorm.hip", r"hipLaunchKernelGGL\(bn_stats_kernel<T>.*?;\n"),
    "bn_final": ("bnorm.hip", r"hipLaunchKernelGGL\(bn_(?:stats|bwd)_final_kernel.*?;\n"),
    "bn_reduce": ("bnorm.hip", r"hipLaunchKernelGGL\(red,.*?;\n"),
    "bn_apply": ("bnorm.hip", r"hipLaunchKernelGGL\(k, dim3\(grid_elem\(n4g, NG\), NG\).*?;\n"),
    "conv_fwd": ("conv.hip", r"    return run\(d, MODE_FWD,.*?;\n"),
    "conv_dgrad": ("conv.hip", r"    return run\(d, MODE_DGRAD,.*?;\n"),
    "conv_wgrad": ("conv.hip", r"    return run\(d, MODE_WGRAD,.*?;\n"),
    "pad_fwd": ("decoder.hip", r"hipLaunchKernelGGL\(k, dim3\(grid_for\(n / 4\)\).*?;\n"),
    "pad_bwd": ("decoder.hip", r"hipLaunchKernelGGL\(k, dim3\(G\).*?;\n"),
    "pool": ("pool.hip", r"hipLaunchKernelGGL\(k, dim3\((?:grid_for\(n\)|\(p\.W).*?;\n"),
    "photo_bwd": ("md2hot.hip", r"hipLaunchKernelGGL\(\(photo_bwd_kernel<NS, SSIM, MASK>\).*?;\n"),
}


def patch(src: str, pattern: str) -> str:
    n = 0

    def twice(m):
        nonlocal n
        n += 1
        stmt = m.group(0)
        if stmt.lstrip().startswith("return "):   # run() whose rc is returned: issue it once before
            first = stmt.replace("return ", "", 1)
            return first + stmt
        return stmt + stmt
    out = re.sub(pattern, twice, src, flags=re.S)
    if n == 0:
        raise SystemExit(f"pattern {pattern!r} not found")
    return out


def main():
    kinds = sys.argv[1:]
    if not kinds or any(k not in KINDS for k in kinds):
        raise SystemExit(f"usage: dup_probe.py KIND [KIND ...]; kinds: {', '.join(KINDS)}")
    for kind in kinds:
        src_name, pattern = KINDS[kind]
        with open(os.path.join(CSRC, src_name)) as f:
            text = patch(f.read(), pattern)
        out_dir = os.path.join(REPO, "abx", "dup_" + kind, "src")
        os.makedirs(out_dir, exist_ok=True)
        src_path = os.path.join(out_dir, src_name)
        with open(src_path, "w") as f:
            f.write(text)
        # build_variant.sh links the patched object with the in-tree objects of the rest
        env = dict(os.environ, SRC=os.path.relpath(src_path, REPO))
        subprocess.run(["bash", os.path.join(REPO, "tools", "build_variant.sh"), "dup_" + kind, "-I" + CSRC],
                       cwd=REPO, env=env, check=True)


if __name__ == "__main__":
    main()
