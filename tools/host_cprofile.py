"""Python-level host cost of the training step: cProfile over a few steps of the
bench configuration (after warm-up/autotune), top functions by own time.
    python tools/host_cprofile.py [steps] [top]"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import monodepth2_amd  # noqa: F401,E402
import torch  # noqa: E402

from monodepth2_amd.data import synthetic_batch  # noqa: E402
from monodepth2_amd.options import default_options  # noqa: E402
from monodepth2_amd.trainer import Trainer  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    dev = torch.device("cuda", 0)
    opt = default_options(batch_size=12, height=192, width=640, weights_init="scratch", log_dir="/tmp/md2_hp",
                          frame_ids=[0, -1, 1], channels_last=True)
    tr = Trainer(opt, device=dev)
    batch = synthetic_batch(12, 192, 640, opt.frame_ids, 4, seed=1, device=dev, eight_bit=True)
    tr.set_train()
    for _ in range(8):
        tr.train_step(batch)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        tr.train_step(batch)
    host = (time.perf_counter() - t) / steps
    torch.cuda.synchronize()
    print(f"host enqueue {1e3 * host:.2f} ms/step (no profiler)")
    if os.environ.get("MD2_SERIAL_BACKWARD"):
        # run the backward on this thread so that cProfile sees its Python code
        torch.autograd.set_multithreading_enabled(False)
        t = time.perf_counter()
        for _ in range(steps):
            tr.train_step(batch)
        torch.cuda.synchronize()
        print(f"serial backward: {1e3 * (time.perf_counter() - t) / steps:.2f} ms/step (incl. GPU)")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        tr.train_step(batch)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats(os.environ.get("MD2_SORT", "tottime")).print_stats(top)


if __name__ == "__main__":
    main()
