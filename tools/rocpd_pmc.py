"""Per-kernel average PMC counter values from rocprofv3 sqlite output (run_results.db):
python tools/rocpd_pmc.py <db> [name-regex]"""
import collections
import re
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    q = """select s.string, p.name, e.event_id, sum(e.value)
           from rocpd_pmc_event e join rocpd_info_pmc p on e.pmc_id = p.id
           join rocpd_kernel_dispatch k on k.event_id = e.event_id
           join rocpd_info_kernel_symbol ks on ks.id = k.kernel_id
           join rocpd_string s on s.id = ks.kernel_name_id
           group by e.event_id, p.name"""
    try:
        rows = list(c.execute(q))
    except sqlite3.OperationalError:
        q = q.replace("s.string", "ks.kernel_name").replace("join rocpd_string s on s.id = ks.kernel_name_id", "")
        rows = list(c.execute(q))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for kname, cname, _, v in rows:
        if rx and not rx.search(kname):
            continue
        agg[kname[:90]][cname].append(v)
    for k, d in agg.items():
        print(k, {n: round(sum(v) / len(v), 1) for n, v in sorted(d.items())}, "n", max(len(v) for v in d.values()))


if __name__ == "__main__":
    main()
