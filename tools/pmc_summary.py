"""Summarise rocprofv3 --pmc counter CSVs: per-counter mean over the steady-state launches of one kernel.

    python tools/pmc_summary.py gpurun_out/<tag>   (every run_counter_collection.csv below it)
"""
import collections
import csv
import glob
import os
import sys


def main(root):
    out = {}
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        rows = list(csv.DictReader(open(f)))
        per = collections.defaultdict(dict)
        dur = {}
        for r in rows:
            d = int(r["Dispatch_Id"])
            per[r["Counter_Name"]][d] = per[r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
            dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for k, v in per.items():
            vals = [v[d] for d in sorted(v)][1:] or list(v.values())   # drop the first (cold) launch
            out[k] = sum(vals) / len(vals)
        ds = [dur[d] for d in sorted(dur)][1:] or list(dur.values())
        out.setdefault("kernel_us", sum(ds) / len(ds))
    for k, v in out.items():
        print(f"{k:32s} {v:16.1f}")
    return out


if __name__ == "__main__":
    main(sys.argv[1])
