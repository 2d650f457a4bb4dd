"""Pinned convolution choices (conv_ops.load_choices / MD2_CONV_CHOICES): with a table,
every process runs the same kernel for every conv shape (no per-process timing), so
training is bitwise reproducible across processes — which the per-process autotune
alone does not guarantee (two processes may time different winners)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STEP = r'''
import os, sys, json
sys.path.insert(0, {repo!r})
import monodepth2_amd
import torch
from monodepth2_amd import conv_ops
from monodepth2_amd.data import synthetic_batch
from monodepth2_amd.options import default_options
from monodepth2_amd.trainer import Trainer
torch.manual_seed(0)
tr = Trainer(default_options(batch_size=2, height=64, width=128, weights_init="scratch", log_dir="/tmp/md2_pin"),
             device=torch.device("cuda", 0))
batch = synthetic_batch(2, 64, 128, tr.opt.frame_ids, 4, seed=3, device="cuda", eight_bit=True)
tr.noise_override = {{s: torch.zeros(*tr.hot.noise_shape(s), device="cuda") for s in range(4)}}
tr.set_train()
for _ in range(2):
    tr.train_step(batch)
torch.cuda.synchronize()
out = sys.argv[1]
if len(sys.argv) > 2:
    conv_ops.save_choices(sys.argv[2])
torch.save([p.detach().cpu() for p in tr.nets.parameters()], out)
print(json.dumps({{"timed": len(conv_ops._times), "choices": len(conv_ops._choice)}}))
'''


def _run(tmp_path, tag, env_extra, save_table=None):
    script = tmp_path / "step.py"
    script.write_text(STEP.format(repo=REPO))
    env = dict(os.environ, **env_extra)
    args = [sys.executable, str(script), str(tmp_path / f"{tag}.pt")] + ([str(save_table)] if save_table else [])
    r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_pinned_choices_reproduce_bitwise_across_processes(tmp_path):
    import torch
    table = tmp_path / "choices.json"
    info = _run(tmp_path, "auto", {}, save_table=table)
    assert info["timed"] > 0 and table.exists()
    rows = json.loads(table.read_text())["rows"]
    assert len(rows) == info["choices"]
    a = _run(tmp_path, "pin_a", {"MD2_CONV_CHOICES": str(table)})
    b = _run(tmp_path, "pin_b", {"MD2_CONV_CHOICES": str(table)})
    assert a["timed"] == 0 and b["timed"] == 0          # nothing timed: every shape pinned
    pa = torch.load(tmp_path / "pin_a.pt", weights_only=True)
    pb = torch.load(tmp_path / "pin_b.pt", weights_only=True)
    assert all(torch.equal(x, y) for x, y in zip(pa, pb))
