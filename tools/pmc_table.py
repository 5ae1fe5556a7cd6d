"""Average per dispatch of every counter in rocprofv3 --pmc output directories.

    python tools/pmc_table.py DIR [DIR ...] [--json OUT]

Each DIR holds one pass (tools/pmc_groups.sh writes p1, p2, ...); the table has one row
per kernel and one column per counter, averaged over that kernel's dispatches, plus the
average duration from the pass's kernel trace when one was collected.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def kname(s):
    return s.split("(")[0].replace("void ", "").strip()


def load(dirs):
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> per-dispatch values
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            for row in csv.DictReader(open(f)):
                per[(kname(row["Kernel_Name"]), row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
            for (k, _, c), v in per.items():
                vals[k][c].append(v)
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                vals[kname(row["Kernel_Name"])]["dur_us"].append(
                    (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}


def main():
    args = sys.argv[1:]
    out = None
    if "--json" in args:
        i = args.index("--json")
        out = args[i + 1]
        args = args[:i] + args[i + 2:]
    tab = load(args)
    for k in sorted(tab):
        print(k)
        for c, v in sorted(tab[k].items()):
            print(f"    {c:40s} {v:16.4g}")
    if out:
        json.dump(tab, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
