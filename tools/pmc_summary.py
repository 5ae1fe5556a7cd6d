"""Summarise rocprofv3 --pmc CSVs: per-kernel mean of each counter, and HBM bytes per
launch of k_window_f corrected with the calibration kernels (tools/pmc_calib.hip).

    python tools/pmc_summary.py gpurun_out/pmc_* > profiles/<round>/pmc_summary.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CALIB_BYTES = 1 << 30


def load(dirs):
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(path)):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                short = name.split("(")[0].split("<")[0].strip()
                if short.startswith("void "):
                    short = short[5:]
                if "k_calib_read" in name or "k_calib_write" in name or "k_calib_gather" in name:
                    short = name.split("(")[0].strip()
                vals[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    vals = load(sys.argv[1:])
    out = {"kernels": {}}
    for k, cs in vals.items():
        out["kernels"][k] = {c: sum(v) / len(v) for c, v in cs.items()}
    cal = {}
    for k, cs in out["kernels"].items():
        for width, tag in (("unsigned char", "r1"), ("unsigned int", "r4"),
                           ("unsigned long", "r8"), ("uint4", "r16")):
            if k.startswith("void k_calib_read<" + width) and "FETCH_SIZE" in cs:
                cal[tag] = cs["FETCH_SIZE"] * 1024 / CALIB_BYTES
        if k.startswith("void k_calib_write<unsigned int") and "WRITE_SIZE" in cs:
            cal["w4"] = cs["WRITE_SIZE"] * 1024 / CALIB_BYTES
        if k.startswith("void k_calib_write<uint4") and "WRITE_SIZE" in cs:
            cal["w16"] = cs["WRITE_SIZE"] * 1024 / CALIB_BYTES
        for tag, name in (("0", "g8_8MB"), ("1", "g8_1GB")):  # 2^25 random 8-B gathers
            if k.startswith("void k_calib_gather<" + tag) and "FETCH_SIZE" in cs:
                cal[name] = cs["FETCH_SIZE"] * 1024 / (8 << 25)
            if k.startswith("void k_calib_gather<" + tag) and "TCC_MISS_sum" in cs:
                cal[name + "_miss_per_gather"] = cs["TCC_MISS_sum"] / (1 << 25)
    out["calibration_counter_per_byte"] = cal
    win = out["kernels"].get("k_window_f", {})
    if "FETCH_SIZE" in win and "WRITE_SIZE" in win and cal:
        # k_window_f reads 8 B/lane (ts, oid) and 4 B/lane (sym, v0, v1) streams: use
        # the 8-byte read calibration; its writes are 4 B/lane
        rd = win["FETCH_SIZE"] * 1024 / cal.get("r8", 1.0)
        wr = win["WRITE_SIZE"] * 1024 / cal.get("w4", 1.0)
        out["k_window_f_hbm_bytes"] = {"read": rd, "write": wr, "total": rd + wr}
    json.dump(out, sys.stdout, indent=1)
    n_ops = int(os.environ.get("SMX_PMC_NOPS", "0"))
    if n_ops and "k_window_f_hbm_bytes" in out:
        # the per-launch HBM bytes bench.py reports as roofline.traffic
        hb = out["k_window_f_hbm_bytes"]
        rec = {"n_ops": n_ops, "kernel": "k_window_f",
               "hbm_bytes_per_launch": round(hb["total"]),
               "read_bytes": round(hb["read"]), "write_bytes": round(hb["write"]),
               "correction": "FETCH_SIZE / calibrated 8-B read factor, WRITE_SIZE / 4-B write "
                             "factor (tools/pmc_calib.hip; MI355X_MICROARCH.md HBM section)"}
        with open(os.environ.get("SMX_PMC_OUT", "pmc_window.json"), "w") as fh:
            json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
