"""GPU busy / idle from a rocprofv3 kernel_trace.csv: the trace is split into windows at idle gaps
longer than --split ms (tools/c5_timeline.py sleeps 1 s between its modes); per window: span, kernel
count, busy (union of kernel intervals), idle fraction and the largest gaps.
    python tools/trace_gaps.py <run_kernel_trace.csv> [--split 200] [--min-kernels 100]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--split", type=float, default=200.0)
    ap.add_argument("--min-kernels", type=int, default=100)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    windows, cur = [], [ks[0]]
    for k in ks[1:]:
        if (k[0] - max(e for _, e, _ in cur[-50:])) / 1e6 > a.split:
            windows.append(cur)
            cur = []
        cur.append(k)
    windows.append(cur)
    for w in windows:
        if len(w) < a.min_kernels:
            continue
        t0, t1 = w[0][0], max(e for _, e, _ in w)
        busy, end, gaps = 0, t0, []
        for s, e, n in w:
            if s > end:
                gaps.append(((s - end) / 1e3, n[:60]))
            busy += max(0, e - max(s, end))
            end = max(end, e)
        span = (t1 - t0) / 1e3
        gaps.sort(reverse=True)
        print(f"window: {len(w)} kernels, span {span:.1f} us, busy {busy / 1e3:.1f} us, idle {1 - busy / 1e3 / span:.3f}, "
              f"gaps > 5 us: {sum(1 for g in gaps if g[0] > 5)} totalling {sum(g[0] for g in gaps if g[0] > 5):.1f} us")
        for g, n in gaps[:5]:
            print(f"   gap {g:8.1f} us before {n}")


if __name__ == "__main__":
    main()
