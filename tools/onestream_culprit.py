"""Which freed eager-pool block does the one-stream captured step (--pose_streams 0) still
read?  After the capture, every free block of the caching allocator is filled with NaN
bytes one at a time (hipMemset on memory the allocator owns but has not handed out) and
the step replayed: a block whose fill makes the gradients non-finite is one the graph
reads; its allocation stack (memory history) names the tensor.
    MD2_ALLOW_ONESTREAM_GRAPH=1 python tools/onestream_culprit.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from monodepth2_amd.data import synthetic_batch  # noqa: E402
from monodepth2_amd.options import default_options  # noqa: E402
from monodepth2_amd.trainer import Trainer  # noqa: E402


def main():
    torch.cuda.memory._record_memory_history(max_entries=200000)
    torch.manual_seed(0)
    tr = Trainer(default_options(batch_size=2, height=64, width=128, weights_init="scratch", log_dir="/tmp/md2_oc",
                                 frame_ids=[0, -1, 1], amp="none", hip_graph=True, pose_streams=0),
                 device=torch.device("cuda", 0))
    batch = synthetic_batch(2, 64, 128, tr.opt.frame_ids, 4, seed=3, device="cuda", eight_bit=True)
    tr.train_step(batch)
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    snap = torch.cuda.memory._snapshot()
    free = []
    for seg in snap["segments"]:
        for blk in seg["blocks"]:
            if blk["state"] == "inactive":
                free.append((blk["address"], blk["size"], seg.get("stream"), seg.get("segment_pool_id"),
                             blk.get("frames", [])))
    print("free blocks: %d" % len(free), flush=True)

    def finite():
        return all(bool(torch.isfinite(p.grad).all()) for p in tr.nets.parameters() if p.grad is not None)

    tr.train_step(batch)
    torch.cuda.synchronize()
    print("baseline replay finite: %s" % finite(), flush=True)
    hits = 0
    for addr, size, stream, pool, frames in free:
        if hip.hipMemset(ctypes.c_void_p(addr), 0xFF, ctypes.c_size_t(size)) != 0:
            continue
        torch.cuda.synchronize()
        tr.train_step(batch)
        torch.cuda.synchronize()
        if not finite():
            hits += 1
            print("HIT block 0x%x size %d stream %s pool %s" % (addr, size, stream, pool), flush=True)
            for f in frames[:25]:
                fn = f.get("filename", "")
                if "monodepth2_amd" in fn or "tools/" in fn or "torch/cuda" in fn or "autograd" in fn:
                    print("     %s:%s %s" % (fn, f.get("line"), f.get("name")), flush=True)
            # a clean state for the next probe: zero the block, replay until finite again
            hip.hipMemset(ctypes.c_void_p(addr), 0, ctypes.c_size_t(size))
            torch.cuda.synchronize()
            with torch.no_grad():
                for p in tr.nets.parameters():
                    if not bool(torch.isfinite(p).all()):
                        p.zero_()
            if hits >= 4:
                break
    print("done: %d hits over %d free blocks" % (hits, len(free)), flush=True)


if __name__ == "__main__":
    main()
