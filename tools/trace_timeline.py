"""Timeline statistics of a rocprofv3 kernel trace (csv output):

    python tools/trace_timeline.py <kernel_trace.csv> [--last-frac 0.5] [--steps N]

Over the last fraction of the trace (the timed steps): wall span, kernel count,
busy time (union of kernel intervals over all queues), the idle gaps between
consecutive busy intervals (count, sum, median), and the time with >= 2 kernels
in flight (overlap of the trainer's two streams).  Used to compare eager and
hipGraph-replayed steps."""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last-frac", type=float, default=0.5)
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    ap.add_argument("--marker", default="", help="kernel-name substring launched once per step: the "
                    "window is from its --skip-th occurrence to its (--skip + --steps)-th")
    ap.add_argument("--skip", type=int, default=0)
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"),
                         r["Kernel_Name"]))
    rows.sort()
    if args.marker:
        marks = [s for s, _, _, n in rows if args.marker in n]
        a, b = marks[args.skip], marks[args.skip + args.steps]
        rows = [r for r in rows if a <= r[0] < b]
    else:
        t0, t1 = rows[0][0], max(r[1] for r in rows)
        cut = t1 - (t1 - t0) * args.last_frac
        rows = [r for r in rows if r[0] >= cut]
    span = max(r[1] for r in rows) - rows[0][0]
    # union of intervals and gaps
    busy, gaps, over = 0, [], 0
    cs, ce = rows[0][0], rows[0][1]
    ev = []
    for s, e, _, _ in rows:
        ev.append((s, 1))
        ev.append((e, -1))
        if s > ce:
            busy += ce - cs
            gaps.append(s - ce)
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    ev.sort()
    depth, last = 0, ev[0][0]
    for t, d in ev:
        if depth >= 2:
            over += t - last
        depth += d
        last = t
    queues = sorted({q for _, _, q, _ in rows})
    n = max(args.steps, 1)
    print(f"kernels {len(rows)} ({len(rows) / n:.0f}/step), queues {queues}")
    print(f"span {span / 1e6 / n:.3f} ms/step, busy {busy / 1e6 / n:.3f} ms/step, "
          f"idle {(span - busy) / 1e6 / n:.3f} ms/step in {len(gaps) / n:.0f} gaps/step "
          f"(median {statistics.median(gaps) / 1e3 if gaps else 0:.2f} us)")
    print(f"two or more kernels in flight: {over / 1e6 / n:.3f} ms/step")
    kern = sum(e - s for s, e, _, _ in rows)
    print(f"summed kernel time {kern / 1e6 / n:.3f} ms/step")


if __name__ == "__main__":
    main()
