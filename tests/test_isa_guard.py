"""The built library's gfx950 code holds no packed-fp32 VALU op whose src1 op_sel has
the low lane read the high dword of its register pair (`v_pk_*_f32 ... op_sel:[x,1...]`).

The disparity-head weight-gradient kernel had exactly four such v_pk_fma_f32 per
instantiation (taps 1 and 7: dz broadcast from the high half of a ds_read2 pair), and
exactly those four accumulators came out intermittently different (low lane only, a
whole wave's worth) while a second process shared the GPU; with the encoding gone the
same runs are bitwise repeatable (tools/determinism_probe.py).  The
sources that produced it are built without SLP vectorisation (build.py FLAGS); this test
keeps the encoding from coming back through any source."""
import os
import re
import shutil
import subprocess

import pytest

from monodepth2_amd import build

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
PATTERN = re.compile(r"v_pk_\w+_f32\s.*op_sel:\[[01],1")


def _device_disassembly(tmp_path):
    lib = build.build()
    local = tmp_path / os.path.basename(lib)
    shutil.copy(lib, local)
    subprocess.run([OBJDUMP, "--offloading", str(local)], cwd=tmp_path, check=True, capture_output=True)
    objs = sorted(p for p in tmp_path.iterdir() if p.name.endswith("gfx950"))
    assert objs, "no gfx950 code object in the library"
    for p in objs:
        out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(p)], check=True, capture_output=True,
                             text=True).stdout
        yield p.name, out


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="ROCm llvm-objdump not present")
def test_no_src1_high_half_packed_fp32(tmp_path):
    bad, kernel, n_pk = [], None, 0
    for name, text in _device_disassembly(tmp_path):
        for line in text.splitlines():
            if line.endswith(">:"):
                kernel = line.split("<", 1)[-1][:-2]
            elif "v_pk_" in line:
                n_pk += 1
                if PATTERN.search(line):
                    bad.append((kernel, line.strip()[:90]))
    assert n_pk > 0, "disassembly found no packed ops at all: the scan is not looking at device code"
    assert not bad, bad[:8]
