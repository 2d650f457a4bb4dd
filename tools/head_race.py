"""Repeat md2_disp_head_bwd on fixed inputs and compare every result bitwise with the
first (the DDP test's intermittent dispconv weight-gradient mismatch,
tools/determinism_probe.py).  Shapes: the four heads of a B=2 64x128 step.

    python tools/head_race.py [--iters 2000] [--procs 2]
"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


FILL = os.environ.get("HEAD_RACE_FILL", "1") == "1"


def worker(rank, iters, out):
    import torch
    from monodepth2_amd import _lib
    L = _lib.lib()
    st = _lib.stream(torch.device("cuda", 0))
    g = torch.Generator(device="cuda").manual_seed(rank)
    CL = torch.channels_last
    res = []
    for C, h, w in [(16, 64, 128), (32, 32, 64), (64, 16, 32), (128, 8, 16)]:
        B = 2
        P = torch.randn(B, C, h + 2, w + 2, device="cuda", generator=g).contiguous(memory_format=CL)
        weight = (torch.randn(1, C, 3, 3, device="cuda", generator=g) * 0.05).contiguous(memory_format=CL)
        disp = torch.rand(B, 1, h, w, device="cuda", generator=g)
        gd = torch.randn(B, 1, h, w, device="cuda", generator=g)
        d = _lib.HeadDesc(B, C, h, w, _lib.HEAD_WEIGHT_CL)
        ws = torch.empty(L.md2_disp_head_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device="cuda")
        ref = None
        cnt = torch.zeros(3, dtype=torch.int64, device="cuda")
        worst = torch.zeros((), device="cuda")
        for it in range(iters):
            gP = torch.empty_like(P, memory_format=CL)
            gw = torch.empty_like(weight)
            gb = torch.empty(1, device="cuda")
            if FILL:   # fresh workspace contents each call, as a new allocation in the step has
                ws.random_(0, 256, generator=g)
                gw.normal_(generator=g)
                gP.normal_(generator=g)
            _lib.check(L.md2_disp_head_bwd(ctypes.byref(d), P.data_ptr(), weight.data_ptr(), disp.data_ptr(),
                                           gd.data_ptr(), gP.data_ptr(), gw.data_ptr(), gb.data_ptr(), ws.data_ptr(),
                                           st), "md2_disp_head_bwd")
            if ref is None:
                ref = (gP.clone(), gw.clone(), gb.clone())
                continue
            # every iteration, on the device (no host sync in the loop)
            cnt[0] += (gP.view(torch.int32) != ref[0].view(torch.int32)).any()
            cnt[1] += (gw.view(torch.int32) != ref[1].view(torch.int32)).any()
            cnt[2] += (gb.view(torch.int32) != ref[2].view(torch.int32)).any()
            worst = torch.maximum(worst, (gw - ref[1]).abs().max())
        torch.cuda.synchronize()
        bad = [int(v) for v in cnt]
        res.append((C, bad))
        print(f"rank {rank} C={C} {h}x{w}: iterations differing from the first (gP, gw, gb): {bad} of {iters - 1}, "
              f"max |dgw| {float(worst):.3e}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--procs", type=int, default=2)
    a = ap.parse_args()
    import torch.multiprocessing as mp
    if a.procs == 1:
        worker(0, a.iters, None)
    else:
        mp.spawn(worker, args=(a.iters, None), nprocs=a.procs, join=True)


if __name__ == "__main__":
    main()
