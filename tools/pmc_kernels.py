"""Per-kernel summary of rocprofv3 --pmc counter CSVs (every *counter_collection.csv below a directory).

    python tools/pmc_kernels.py gpurun_out/<tag> [kernel-substring ...]

For each kernel name: launches, mean duration, the mean of every counter over its launches (the
first launch of each kernel dropped as cold), and the derived figures the DESIGN tables quote:
clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE
/ 8 x 1024 SIMDs); FETCH_SIZE / WRITE_SIZE in KB per launch (MI355X_MICROARCH.md rocprofv3 section).
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*\)$", "", name.strip())
    name = re.sub(r"^void ", "", name)
    return name.replace("cn::mlp::", "").replace("cn::", "")


def main(root, subs=()):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    dur = collections.defaultdict(dict)
    gdur = collections.defaultdict(dict)   # durations of the launches GRBM_GUI_ACTIVE was read on
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if subs and not any(s in k for s in subs):
                continue
            key = (f, int(r["Dispatch_Id"]))
            per[k][r["Counter_Name"]][key] = per[k][r["Counter_Name"]].get(key, 0.0) + float(r["Counter_Value"])
            dur[k][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                gdur[k][key] = dur[k][key]
    out = {}
    for k in per:
        row = {}
        for c, v in per[k].items():
            vals = [v[d] for d in sorted(v)]
            vals = vals[1:] if len(vals) > 1 else vals
            row[c] = sum(vals) / len(vals)
        ds = [dur[k][d] for d in sorted(dur[k])]
        ds = ds[1:] if len(ds) > 1 else ds
        row["kernel_us"] = sum(ds) / len(ds)
        row["launches"] = len(ds)
        if "GRBM_GUI_ACTIVE" in row:
            cyc = row["GRBM_GUI_ACTIVE"] / 8.0
            gd = [gdur[k][d] for d in sorted(gdur[k])]
            gd = gd[1:] if len(gd) > 1 else gd
            row["kernel_us_grbm_pass"] = sum(gd) / len(gd)
            row["clock_ghz"] = cyc / (row["kernel_us_grbm_pass"] * 1e3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in row:
                row["mfma_busy"] = row["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)
        if "SQ_WAVE_CYCLES" in row and row["SQ_WAVE_CYCLES"]:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in row:
                    row[c + "_frac"] = row[c] / row["SQ_WAVE_CYCLES"]
        out[k] = row
    for k, row in sorted(out.items()):
        print(k)
        for c, v in sorted(row.items()):
            print(f"    {c:32s} {v:18.4f}" if isinstance(v, float) and abs(v) < 100 else f"    {c:32s} {v:18.1f}")
    return out


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
