"""Fold the GPU run's margin lines (tests/conftest.py::margin, CN_MARGINS=<path>.jsonl) into one JSON:
every (test, quantity) with its observed error, its bound and their ratio, sorted by ratio, plus a
summary (how many, the tightest).     python tools/margins_json.py <in.jsonl> <out.json> [--source TEXT]"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--source", default="")
    args = ap.parse_args()
    rows = [json.loads(line) for line in open(args.src) if line.strip()]
    rows.sort(key=lambda r: -(r.get("ratio") or 0.0))
    ratios = [r["ratio"] for r in rows if r.get("ratio") is not None]
    out = {
        "source": args.source,
        "n": len(rows),
        "tests": len({r["test"] for r in rows}),
        "max_ratio": max(ratios) if ratios else None,
        "n_ratio_over_half": sum(x > 0.5 for x in ratios),
        "exact": sum(r["err"] == 0.0 for r in rows),
        "margins": rows,
    }
    with open(args.dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "margins"}))


if __name__ == "__main__":
    main()
