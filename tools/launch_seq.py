"""One steady iteration's launch sequence from a rocprofv3 kernel trace: every kernel between the
(k-1)-th and k-th occurrence of an anchor kernel (default: the forward field kernel that starts an
iteration), with its duration and the idle gap before it -- which launches are coarse / fine, how long
each takes, and how much of the iteration the GPU sits idle.
    python tools/launch_seq.py <run_kernel_trace.csv> [--anchor NAME] [--per-iter N] [--iter K]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--anchor", default="field_w16_kernel<", help="substring of the kernel that recurs per_iter times")
    ap.add_argument("--per-iter", type=int, default=8, help="anchor launches per iteration")
    ap.add_argument("--iter", type=int, default=-3, help="which iteration (python index over whole iterations)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.anchor in r["Kernel_Name"]]
    starts = idx[::a.per_iter]
    its = list(zip(starts[:-1], starts[1:]))
    lo, hi = its[a.iter]
    prev_end = None
    busy = 0.0
    t0 = int(rows[lo]["Start_Timestamp"])
    for r in rows[lo:hi]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = 0.0 if prev_end is None else (s - prev_end) / 1e3
        busy += (e - s) / 1e3
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:6.1f}  grid {r['Grid_Size_X']:>7s}  "
              f"{r['Kernel_Name'][:90]}")
        prev_end = e
    span = (int(rows[hi]["Start_Timestamp"]) - t0) / 1e3
    print(f"iteration span {span:.1f} us, kernels busy {busy:.1f} us ({busy / span:.4f}), {hi - lo} launches")


if __name__ == "__main__":
    main()
