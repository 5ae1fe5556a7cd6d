"""Per-kernel average durations (us) from rocprofv3 SQLite outputs (rocpd *.db), one
column per run: python tools/rocpd_stats.py name=path.db ... [--last K]"""
import argparse
import collections
import sqlite3


def kernel_times(path, last):
    c = sqlite3.connect(path)
    q = ("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    agg = collections.defaultdict(list)
    for name, a, b in c.execute(q):
        agg[name.split("(")[0].replace("void ", "")].append((b - a) / 1e3)
    return {k: sum(v[-last:]) / len(v[-last:]) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--last", type=int, default=5, help="average the last K calls of each kernel")
    ap.add_argument("runs", nargs="+")
    a = ap.parse_args()
    cols = {}
    for r in a.runs:
        name, path = r.split("=", 1)
        cols[name] = kernel_times(path, a.last)
    first = next(iter(cols.values()))
    print("%-40s" % "kernel (avg us, last %d calls)" % a.last, *["%9s" % n for n in cols])
    for k in sorted(first, key=lambda k: -first[k]):
        print("%-40s" % k[:40], *[("%9.1f" % c[k]) if k in c else "%9s" % "-" for c in cols.values()])


if __name__ == "__main__":
    main()
