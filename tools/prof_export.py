"""Export the per-kernel summary of a rocprofv3 --kernel-trace --stats database to CSV.

    python tools/prof_export.py gpurun_out/prof4 profiles/r06_final/kernel_stats.csv
"""
import csv
import glob
import sqlite3
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    db = glob.glob(f"{src}/**/*.db", recursive=True)[0]
    con = sqlite3.connect(db)
    rows = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for r in rows:
            w.writerow([r[0], r[1], round(r[2], 1), round(r[3], 1), round(r[4], 3)])


if __name__ == "__main__":
    main()
