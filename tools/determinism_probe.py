"""Which op of a training step is not bitwise repeatable?

Runs the Trainer's process_batch + backward N times on one batch (the setting of
tests/test_distributed_gpu.py: B=2, 64x128, scratch weights) and compares, pass by
pass against pass 0, every convolution's forward output, every convolution's
backward inputs / outputs (gy, gx, gw), the disparities, the losses and every
parameter gradient — bitwise, in call order.  The first differing tensor names the
nondeterministic op.  Every conv choice (per op and shape, the candidate name) is
logged with it.

  python tools/determinism_probe.py --passes 4 [--world 2 --backend gloo] [--autotune 0|1]
                                    [--deterministic 0|1] --out gpurun_out/det

With --world 2 two processes share cuda:0 over gloo and the passes alternate
no_sync / synced DDP backward, as the distributed test does.
"""
import argparse
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Recorder:
    def __init__(self):
        self.passes = []
        self.cur = None

    def start(self):
        self.cur = []
        self.passes.append(self.cur)

    def add(self, name, t):
        # a device copy now (no host sync inside the step: the step keeps its timing),
        # moved to the host once the pass is done (finish)
        if self.cur is not None and torch.is_tensor(t):
            self.cur.append((name, t.detach().clone()))

    def finish(self):
        torch.cuda.synchronize()
        if self.cur is not None:
            self.cur[:] = [(n, t.float().cpu()) for n, t in self.cur]


def _install(rec, conv_ops):
    orig_apply = conv_ops._Conv.apply
    orig_bwd = conv_ops._Conv.backward
    counter = {"f": 0, "b": 0}

    def apply(x, w, stride, pad):
        y = orig_apply(x, w, stride, pad)
        i = counter["f"]
        counter["f"] += 1
        key = (tuple(x.shape), tuple(w.shape), stride, pad)
        ch = conv_ops._choice.get(("fwd",) + key)
        nm = conv_ops._names.get(("fwd",) + key)
        rec.add("fwd#%d %s %s" % (i, key, nm[ch] if (nm and ch is not None) else ch), y)
        return y

    def backward(ctx, gy):
        i = counter["b"]
        counter["b"] += 1
        rec.add("bwd#%d gy %s" % (i, ctx.key), gy)
        gx, gw, a, b = orig_bwd(ctx, gy)
        d = {}
        for op in ("dgrad", "wgrad"):
            ch = conv_ops._choice.get((op,) + ctx.key)
            nm = conv_ops._names.get((op,) + ctx.key)
            d[op] = nm[ch] if (nm and ch is not None) else ch
        rec.add("bwd#%d gx %s %s" % (i, ctx.key, d["dgrad"]), gx)
        rec.add("bwd#%d gw %s %s" % (i, ctx.key, d["wgrad"]), gw)
        return gx, gw, a, b

    conv_ops._Conv.apply = staticmethod(apply)
    conv_ops._Conv.backward = staticmethod(backward)

    # the disparity heads: their input P at the forward, and again (its memory as it
    # is then) with dL/ddisp, disp and the outputs at the backward
    from monodepth2_amd import decoder_ops
    H = decoder_ops._DispHead
    hf, hb = H.forward, H.backward

    def head_fwd(ctx, P, weight, bias):
        out = hf(ctx, P, weight, bias)
        ctx.probe_id = counter["h"] = counter.get("h", 0) + 1
        rec.add("head%d fwd P" % ctx.probe_id, P)
        ctx.probe_P = P.detach().clone()
        rec.add("head%d fwd disp" % ctx.probe_id, out)
        return out

    def head_bwd(ctx, gdisp):
        P, weight, disp = ctx.saved_tensors
        i = ctx.probe_id
        rec.add("head%d bwd P (memory at the backward)" % i, P)
        rec.add("head%d bwd P - P at its forward" % i, P - ctx.probe_P)
        rec.add("head%d bwd gdisp" % i, gdisp)
        gP, gw, gb = hb(ctx, gdisp)
        # the same call replayed twice right here, on the same inputs, each with a fresh
        # workspace filled with garbage: same inputs -> same bits, or the kernel is not
        import ctypes
        from monodepth2_amd import _lib
        L = _lib.lib()
        g32 = gdisp.float().contiguous()
        for rep in range(2):
            ws = torch.empty(L.md2_disp_head_workspace_bytes(ctypes.byref(ctx.d)), dtype=torch.uint8,
                             device=P.device).random_(0, 256)
            gP2, gw2, gb2 = torch.empty_like(gP), torch.empty_like(gw), torch.empty_like(gb)
            _lib.check(L.md2_disp_head_bwd(ctypes.byref(ctx.d), P.data_ptr(), weight.data_ptr(), disp.data_ptr(),
                                           g32.data_ptr(), gP2.data_ptr(), gw2.data_ptr(), gb2.data_ptr(),
                                           ws.data_ptr(), _lib.stream(P.device)), "md2_disp_head_bwd")
            rec.add("head%d replay%d gw" % (i, rep), gw2)
            rec.add("head%d replay%d gP" % (i, rep), gP2)
            rec.add("head%d replay%d partials" % (i, rep), ws.view(torch.float32))
            # the inputs as the stream sees them right after this replay
            rec.add("head%d replay%d in P" % (i, rep), P)
            rec.add("head%d replay%d in disp" % (i, rep), disp)
            rec.add("head%d replay%d in gdisp" % (i, rep), g32)
        rec.add("head%d bwd gP" % i, gP)
        rec.add("head%d bwd gw" % i, gw)
        rec.add("head%d bwd gb" % i, gb)
        return gP, gw, gb

    H.forward = staticmethod(head_fwd)
    H.backward = staticmethod(head_bwd)
    return counter


def _compare(passes):
    """[(pass, first differing name, max abs diff, n differing among the pass)]"""
    out = []
    base = passes[0]
    for k, p in enumerate(passes[1:], 1):
        first, ndiff, worst = None, 0, []
        if len(p) != len(base):
            out.append({"pass": k, "error": "record count %d vs %d" % (len(p), len(base))})
            continue
        for (n0, t0), (n1, t1) in zip(base, p):
            same = t0.shape == t1.shape and torch.equal(t0, t1)
            if not same:
                ndiff += 1
                md = float((t0 - t1).abs().max()) if t0.shape == t1.shape else float("nan")
                rel = md / (float(t0.abs().max()) + 1e-30)
                worst.append({"name": n1, "name0": n0, "max_abs": md, "rel_max": rel})
                if first is None:
                    first = n1
        out.append({"pass": k, "first_diff": first, "n_diff": ndiff, "of": len(p), "diffs": worst[:40]})
    return out


def _record_outputs(rec, tr, outputs, losses):
    for s in range(4):
        rec.add("disp%d" % s, outputs[("disp", s)])
    for f in tr.src_frames:
        if ("cam_T_cam", 0, f) in outputs:
            rec.add("cam_T_cam %s" % f, outputs[("cam_T_cam", 0, f)])
    for s in range(4):
        if "identity_selection/%d" % s in outputs:
            rec.add("identity_selection/%d" % s, outputs["identity_selection/%d" % s])
    rec.add("loss", losses["loss"])


def run(rank, world, port, args):
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group(args.backend, rank=rank, world_size=world)
    torch.backends.cudnn.deterministic = bool(args.deterministic)
    dev = torch.device("cuda", 0)
    from monodepth2_amd import conv_ops
    from monodepth2_amd.data import synthetic_batch
    from monodepth2_amd.options import default_options
    from monodepth2_amd.trainer import Trainer
    conv_ops.AUTOTUNE = bool(args.autotune)
    rec = Recorder()
    counter = _install(rec, conv_ops)
    torch.manual_seed(0)
    tr = Trainer(default_options(batch_size=2, height=64, width=128, weights_init="scratch",
                                 log_dir="/tmp/md2_det", pose_streams=args.pose_streams), device=dev, rank=rank,
                 world_size=world)
    tr.set_train()
    batch = synthetic_batch(2, 64, 128, tr.opt.frame_ids, 4, seed=10 + rank, device=dev)
    if args.first_step:
        tr.train_step(batch)
        torch.cuda.synchronize()
    params = [(n, p) for n, p in tr.nets.named_parameters() if p.requires_grad and "fc." not in n]
    modes = []
    for k in range(args.passes):
        counter["h"] = 0
        rec.start()
        tr.model_optimizer.zero_grad(set_to_none=True)
        sync = world > 1 and (k % 2 == 1)
        modes.append("synced" if sync else "local")
        if tr.ddp is not None and not sync:
            with tr.ddp.no_sync():
                outputs, losses = tr.process_batch(batch)
                _record_outputs(rec, tr, outputs, losses)
                losses["loss"].backward()
        else:
            outputs, losses = tr.process_batch(batch)
            _record_outputs(rec, tr, outputs, losses)
            losses["loss"].backward()
        torch.cuda.synchronize()
        for n, p in params:
            if p.grad is not None:
                g = p.grad.detach().clone()
                if sync:   # the synced pass holds the mean: compare its local part instead
                    continue
                rec.add("grad " + n, g)
        rec.finish()
        byname = dict(rec.cur)
        for hi in range(1, 5):
            a, r0, r1 = byname.get("head%d bwd gw" % hi), byname.get("head%d replay0 gw" % hi), \
                byname.get("head%d replay1 gw" % hi)
            if a is None:
                continue
            if not (torch.equal(a, r0) and torch.equal(r0, r1)):
                p0, p1 = byname["head%d replay0 partials" % hi], byname["head%d replay1 partials" % hi]
                n = a.numel() + 1   # a partial row: 9·C weight taps + the bias
                rows = (p0 - p1).view(-1, n).abs().amax(1)
                bad = torch.nonzero(rows).flatten().tolist()
                same_in = all(torch.equal(byname["head%d replay0 in %s" % (hi, t)],
                                          byname["head%d replay1 in %s" % (hi, t)]) for t in ("P", "disp", "gdisp"))
                dgp = (byname["head%d replay0 gP" % hi] - byname["head%d replay1 gP" % hi]).abs()
                print("PROBE: inputs identical across the replays: %s; replay gP differing elements %d (max %.3e)"
                      % (same_in, int((dgp != 0).sum()), float(dgp.max())), flush=True)
                for rr in bad[:4]:
                    d = (p0 - p1).view(-1, n)[rr]
                    idx = torch.nonzero(d).flatten().tolist()
                    print("PROBE:   row %d: %d of %d entries differ, first %s, values %s vs %s" % (
                        rr, len(idx), n, idx[:12], p0.view(-1, n)[rr][idx[:4]].tolist(),
                        p1.view(-1, n)[rr][idx[:4]].tolist()), flush=True)
                print("PROBE: pass %d head %d: gw / replay0 / replay1 not all equal: |a-r0| %.3e |r0-r1| %.3e; "
                      "partial rows differing between the replays: %s of %d" % (
                          k, hi, float((a - r0).abs().max()), float((r0 - r1).abs().max()), bad[:20],
                          rows.numel()), flush=True)
        for n, t in rec.cur:
            if n.endswith("P - P at its forward") and float(t.abs().max()) != 0.0:
                print("PROBE: %s nonzero: %d elements, max %.3e (pass %d)" % (n, int((t != 0).sum()),
                                                                             float(t.abs().max()), k), flush=True)
    # compare local passes only among themselves, synced among themselves
    res = {"rank": rank, "world": world, "autotune": args.autotune, "deterministic": args.deterministic,
           "modes": modes}
    loc = [p for p, m in zip(rec.passes, modes) if m == "local"]
    syn = [p for p, m in zip(rec.passes, modes) if m == "synced"]
    res["local_vs_local"] = _compare(loc) if len(loc) > 1 else []
    res["synced_vs_synced"] = _compare(syn) if len(syn) > 1 else []
    if loc and syn:
        # the forward + the backward up to the parameter gradients are the same computation
        n = min(len(loc[0]), len(syn[0]))
        res["local0_vs_synced0"] = _compare([loc[0][:n], syn[0][:n]])
    res["choices"] = {"%s %s" % (k[0], k[1:]): conv_ops._names[k][i] for k, i in conv_ops._choice.items()
                      if k in conv_ops._names}
    os.makedirs(args.out, exist_ok=True)
    with open(os.path.join(args.out, "det%s_w%d_a%d_d%d_r%d.json" % (args.tag, world, args.autotune, args.deterministic, rank)),
              "w") as f:
        json.dump(res, f, indent=1)
    for key in ("local_vs_local", "synced_vs_synced", "local0_vs_synced0"):
        for r in res.get(key, []):
            print("rank %d %s pass %s: first diff %s (%s of %s differ)" % (
                rank, key, r.get("pass"), r.get("first_diff"), r.get("n_diff"), r.get("of")), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=4)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--autotune", type=int, default=1)
    ap.add_argument("--deterministic", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/det")
    ap.add_argument("--first-step", type=int, default=1, help="one train_step first (autotune + agree)")
    ap.add_argument("--tag", default="")
    ap.add_argument("--pose-streams", type=int, default=1, help="0: the pose network on the main stream")
    args = ap.parse_args()
    if args.world == 1:
        run(0, 1, 0, args)
    else:
        mp.spawn(run, args=(args.world, _free_port(), args), nprocs=args.world, join=True)


if __name__ == "__main__":
    main()
