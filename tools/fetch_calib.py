"""Calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE on this GPU for the access widths the
hot-path kernels use (tools/fetch_calib.hip).  Run on the GPU box from the repo root:

    python tools/fetch_calib.py [out.json]

Builds tools/fetch_calib if needed, runs one rocprofv3 --pmc pass per counter, and
prints per kernel: the counter in bytes (KB x 1024), the known bytes the kernel moves,
and known / counted — the factor a counted byte figure of that access width must be
multiplied by (MI355X_MICROARCH.md §HBM: 2.0 for 16 B/lane streaming reads, 1.0 for
16 B/lane streaming stores; the rest is what this measures).
"""
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "tools", "fetch_calib")
MB = 256 << 20
LINES = MB // 128
# (kernel name as rocprof prints it, counter, known bytes, what)
KERNELS = [
    ("read_coalesced<unsigned char>", "FETCH_SIZE", MB, "read 1 B/lane coalesced"),
    ("read_coalesced<unsigned short>", "FETCH_SIZE", MB, "read 2 B/lane coalesced"),
    ("read_coalesced<unsigned int>", "FETCH_SIZE", MB, "read 4 B/lane coalesced"),
    ("read_coalesced<HIP_vector_type<unsigned int, 2u> >", "FETCH_SIZE", MB, "read 8 B/lane coalesced"),
    ("read_coalesced<HIP_vector_type<unsigned int, 4u> >", "FETCH_SIZE", MB, "read 16 B/lane coalesced"),
    ("read_lines<unsigned int>", "FETCH_SIZE", LINES * 128, "gather 4 B per 128-B line (known = whole lines)"),
    ("read_lines<HIP_vector_type<unsigned int, 2u> >", "FETCH_SIZE", LINES * 128,
     "gather 8 B per 128-B line (known = whole lines)"),
    ("write_coalesced<unsigned char>", "WRITE_SIZE", MB, "write 1 B/lane coalesced"),
    ("write_coalesced<unsigned int>", "WRITE_SIZE", MB, "write 4 B/lane coalesced"),
    ("write_coalesced<HIP_vector_type<unsigned int, 2u> >", "WRITE_SIZE", MB, "write 8 B/lane coalesced"),
    ("write_coalesced<HIP_vector_type<unsigned int, 4u> >", "WRITE_SIZE", MB, "write 16 B/lane coalesced"),
]


def run(counter):
    d = tempfile.mkdtemp(prefix="calib_", dir="/tmp")
    cmd = ["rocprofv3", "--pmc", counter, "-d", d, "-o", "calib", "--output-format", "csv", "--", EXE]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, env=dict(os.environ, TMPDIR="/tmp"), timeout=120)
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                name = re.sub(r"^void ", "", r["Kernel_Name"]).split("(")[0]
                vals[name] = vals.get(name, 0.0) + float(r["Counter_Value"])
    shutil.rmtree(d, ignore_errors=True)
    return vals


def main():
    if not os.path.exists(EXE):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-o", EXE, EXE + ".hip"], check=True)
    got = {c: run(c) for c in ("FETCH_SIZE", "WRITE_SIZE")}
    rows = []
    for name, counter, known, what in KERNELS:
        v = got[counter].get(name)
        counted = None if v is None else 1024.0 * v
        rows.append({"kernel": name, "counter": counter, "what": what, "known_bytes": known,
                     "counted_bytes": counted, "factor": None if not counted else round(known / counted, 4)})
        print(f"{what:48s} {counter:10s} counted {counted} known {known} factor {rows[-1]['factor']}")
    out = {"rows": rows, "unknown_kernels": sorted(set(got["FETCH_SIZE"]) - {r["kernel"] for r in rows}),
           "note": "factor = known bytes / counted bytes (KB x 1024); one rocprofv3 --pmc pass per counter"}
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
