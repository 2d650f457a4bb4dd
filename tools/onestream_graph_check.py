"""Does a captured step with the pose network on the main stream (--pose_streams 0)
replay?  Small size; per replay: the loss, whether the parameters moved, the gradient
norm.  MD2_ALLOW_ONESTREAM_GRAPH=1 python tools/onestream_graph_check.py [--pose-streams 0] [--amp none]
(the Trainer refuses --hip_graph with --pose_streams 0 otherwise: the open bug this reproduces)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from monodepth2_amd.data import synthetic_batch  # noqa: E402
from monodepth2_amd.options import default_options  # noqa: E402
from monodepth2_amd.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pose-streams", type=int, default=0)
    ap.add_argument("--amp", default="none")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--quiet", type=int, default=0, help="replays without host-side work between them")
    ap.add_argument("--between", default="none", choices=["none", "gpu", "host"],
                    help="with --quiet: GPU allocations (parameter clones) or host allocations between replays")
    ap.add_argument("--vary", type=int, default=0, help="with --quiet: a new batch every replay")
    a = ap.parse_args()
    torch.manual_seed(0)
    tr = Trainer(default_options(batch_size=a.batch, height=64, width=128, weights_init="scratch",
                                 log_dir="/tmp/md2_os", frame_ids=[0, -1, 1], amp=a.amp, hip_graph=True,
                                 pose_streams=a.pose_streams), device=torch.device("cuda", 0))
    if a.quiet:
        batch = synthetic_batch(a.batch, 64, 128, tr.opt.frame_ids, 4, seed=3, device="cuda", eight_bit=True)
        keep = []
        batches = [synthetic_batch(a.batch, 64, 128, tr.opt.frame_ids, 4, seed=3 + k, device="cuda", eight_bit=True)
                   for k in range(6)] if a.vary else [batch] * 6
        for k in range(6):
            tr.train_step(batches[k])
            if a.between == "gpu":
                keep.append([p.detach().clone() for p in tr.nets.parameters()])
            elif a.between == "host":
                keep.append([bytearray(4096) for _ in range(2000)] + [object() for _ in range(20000)])
        torch.cuda.synchronize()
        bad = [n for n, p in tr.nets.named_parameters() if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
        badp = [n for n, p in tr.nets.named_parameters() if not bool(torch.isfinite(p).all())]
        print("quiet: %d non-finite grads %s; %d non-finite params" % (len(bad), bad[:20], len(badp)), flush=True)
        return
    parts = set(os.environ.get("MD2_OS_PARTS", "batch,clone,norm").split(","))
    batch = synthetic_batch(a.batch, 64, 128, tr.opt.frame_ids, 4, seed=3, device="cuda", eight_bit=True)
    for k in range(6):
        if "batch" in parts:
            batch = synthetic_batch(a.batch, 64, 128, tr.opt.frame_ids, 4, seed=3 + k, device="cuda", eight_bit=True)
        p0 = [p.detach().clone() for p in tr.nets.parameters()] if "clone" in parts else \
            [p.detach() for p in tr.nets.parameters()]
        _, l = tr.train_step(batch)
        torch.cuda.synchronize()
        if "norm" not in parts:
            continue
        moved = sum(int(not torch.equal(p0[i], p.detach())) for i, p in enumerate(tr.nets.parameters()))
        gn = sum(float(p.grad.float().norm()) ** 2 for p in tr.nets.parameters() if p.grad is not None) ** 0.5
        fin = all(bool(torch.isfinite(p).all()) for p in tr.nets.parameters())
        print("step %d loss %.9g params moved %d/%d grad norm %.4g params finite %s" % (
            k, float(l["loss"]), moved, len(p0), gn, fin), flush=True)
        if k == 5:
            for i, (n, p) in enumerate(tr.nets.named_parameters()):
                bad = p.grad is not None and not bool(torch.isfinite(p.grad).all())
                still = torch.equal(p0[i], p.detach())
                if bad or still:
                    print("   %-55s grad finite %s  moved %s  grad ptr %x" % (
                        n, not bad, not still, p.grad.data_ptr() if p.grad is not None else 0), flush=True)

    bad = [n for n, p in tr.nets.named_parameters() if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
    print("final: %d non-finite grads %s" % (len(bad), bad[:12]), flush=True)


if __name__ == "__main__":
    main()
