"""Idle time between kernels in a bench.py rocprofv3 kernel trace (dev tool):
steps delimited as in step_breakdown.py (the fused AdamW kernels); for the
last K steps: wall time per step, kernel time, the sum of gaps between one
kernel's end and the next one's start, and the gap distribution.

    python tools/kgaps.py <t_kernel_trace.csv> [K]"""
import csv
import json
import sys


def main():
    path, k = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    idx = [i for i, (n, _, _) in enumerate(ev) if "adam" in n.lower()]
    ends, prev = [], None
    for i in idx:
        if prev is not None and i - prev > 50:
            ends.append(prev)
        prev = i
    ends.append(prev)
    lo, hi = ends[-k - 1] + 1, ends[-1] + 1
    sel = ev[lo:hi]
    wall = (sel[-1][2] - sel[0][1]) / 1e6 / k
    busy = sum(e - s for _, s, e in sel) / 1e6 / k
    gaps = [max(0, sel[i + 1][1] - sel[i][2]) for i in range(len(sel) - 1)]
    gaps.sort()
    q = lambda f: gaps[int(f * (len(gaps) - 1))] / 1e3  # noqa: E731
    print(json.dumps({"steps": k, "kernels_per_step": len(sel) / k, "wall_ms_per_step": wall,
                      "kernel_ms_per_step": busy, "gap_ms_per_step": sum(gaps) / 1e6 / k,
                      "gap_us_p50": q(0.5), "gap_us_p90": q(0.9), "gap_us_p99": q(0.99),
                      "gaps_over_20us": sum(1 for g in gaps if g > 20000) / k}))


if __name__ == "__main__":
    main()
