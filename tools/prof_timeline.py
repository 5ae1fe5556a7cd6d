"""Print the kernel timeline of the last N dispatches in a rocprofv3 --kernel-trace database:
start offset, duration and the idle gap before each kernel (microseconds).

    python tools/prof_timeline.py gpurun_out/r03_u/prof_c5 60 > profiles/r03_u/c5_timeline.txt
"""
import glob
import sqlite3
import sys


def main():
    src = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    db = glob.glob(f"{src}/**/*.db", recursive=True)[0]
    con = sqlite3.connect(db)
    cur = con.execute("select * from kernels limit 1")
    cols = [d[0] for d in cur.description]
    name = next(c for c in ("name", "kernel_name", "display_name") if c in cols)
    start = next(c for c in cols if c.lower() in ("start", "start_ns", "begin"))
    end = next(c for c in cols if c.lower() in ("end", "end_ns", "stop"))
    rows = con.execute(f"select {name}, {start}, {end} from kernels order by {start}").fetchall()
    rows = rows[-last:]
    t0 = rows[0][1]
    prev_end = None
    print(f"{'start_us':>10} {'dur_us':>8} {'gap_us':>8}  kernel")
    busy = 0
    for n, s, e in rows:
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        busy += e - s
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} {gap:8.1f}  {n.split('(')[0][:60]}")
        prev_end = e if prev_end is None else max(prev_end, e)
    span = (rows[-1][2] - t0) / 1e3
    print(f"span {span:.1f} us, kernels busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
