"""Per-layer MIOpen convolution throughput of the training step's shapes (fp32,
channels_last, FAST find mode with the shipped find-db): forward and forward+backward
time per call and the achieved TFLOP/s.  python tools/conv_table.py [out.json]"""
import json
import sys

import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import monodepth2_amd  # noqa: F401  (MIOpen env: FAST mode + shipped find-db)
from monodepth2_amd import networks


def conv_shapes(B=12, H=192, W=640):
    """(name, batch, cin, cout, k, stride, h_in, w_in) of every conv in one step."""
    out = []
    enc = networks.ResnetEncoder(18, False)
    hooks = []

    def rec(name, bmul):
        def f(m, inp, outp):
            x = inp[0]
            out.append((name, x.shape[0], m.in_channels, m.out_channels, m.kernel_size[0], m.stride[0],
                        x.shape[2], x.shape[3], m.padding[0]))
        return f
    for n, m in enc.named_modules():
        if isinstance(m, torch.nn.Conv2d):
            hooks.append(m.register_forward_hook(rec("enc." + n, 1)))
    with torch.no_grad():
        feats = enc(torch.zeros(B, 3, H, W))
    for h in hooks:
        h.remove()
    dec = networks.DepthDecoder(enc.num_ch_enc, range(4))
    dec.fused = False
    for n, m in dec.named_modules():
        if isinstance(m, torch.nn.Conv2d):
            m.register_forward_hook(rec("dec." + n, 1))
    with torch.no_grad():
        dec(feats)
    return out


def main():
    dev = torch.device("cuda")
    rows = []
    seen = {}
    for (name, b, cin, cout, k, s, h, w, p) in conv_shapes():
        key = (b, cin, cout, k, s, h, w, p)
        if key in seen:
            seen[key]["layers"].append(name)
            continue
        conv = torch.nn.Conv2d(cin, cout, k, s, p, bias=False).to(dev).to(memory_format=torch.channels_last)
        x = torch.randn(b, cin, h, w, device=dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        y = conv(x)
        g = torch.randn_like(y)
        ho, wo = y.shape[2], y.shape[3]
        flops = 2.0 * b * ho * wo * cout * cin * k * k
        for _ in range(3):
            torch.autograd.grad(conv(x), (x, conv.weight), g)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        n = 10
        ev[0].record()
        for _ in range(n):
            conv(x)
        ev[1].record()
        for _ in range(n):
            torch.autograd.grad(conv(x), (x, conv.weight), g)
        ev[2].record()
        torch.cuda.synchronize()
        tf = ev[0].elapsed_time(ev[1]) / n
        tfb = ev[1].elapsed_time(ev[2]) / n
        r = {"layers": [name], "shape": key, "fwd_ms": round(tf, 4), "bwd_ms": round(tfb - tf, 4),
             "fwd_tflops": round(flops / tf / 1e9, 1), "bwd_tflops": round(2 * flops / max(tfb - tf, 1e-6) / 1e9, 1)}
        seen[key] = r
        rows.append(r)
    tot_f = sum(r["fwd_ms"] * len(r["layers"]) for r in rows)
    tot_b = sum(r["bwd_ms"] * len(r["layers"]) for r in rows)
    for r in sorted(rows, key=lambda r: -(r["fwd_ms"] + r["bwd_ms"]) * len(r["layers"])):
        print(f"{(r['fwd_ms'] + r['bwd_ms']) * len(r['layers']):7.3f} ms  fwd {r['fwd_ms']:.3f} ({r['fwd_tflops']:6.1f} TF)"
              f"  bwd {r['bwd_ms']:.3f} ({r['bwd_tflops']:6.1f} TF)  x{len(r['layers'])} {r['shape']} {r['layers'][0]}")
    print(f"total depth-net convs: fwd {tot_f:.3f} ms, bwd {tot_b:.3f} ms")
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
