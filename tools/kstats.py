"""Summarise a rocprofv3 kernel trace (rocpd .db or kernel_trace.csv): per-kernel
totals, or the dispatch sequence of kernels matching a pattern.  Dev tool."""
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:90]


def load(path):
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        return [(n, (e - s) / 1000.0) for n, s, e in
                db.execute("select name, start, end from kernels order by start")]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
            for r in rows]


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else None
    rows = [(short(n), d) for n, d in load(path)]
    if pat:
        for n, d in rows:
            if re.search(pat, n):
                print(f"{n:90s} {d:9.1f}")
        return
    agg = defaultdict(lambda: [0, 0.0])
    for n, d in rows:
        agg[n][0] += 1
        agg[n][1] += d
    tot = sum(v[1] for v in agg.values())
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{n:90s} calls {c:6d} total_us {t:11.1f} avg_us {t / c:9.1f} {100 * t / tot:5.1f}%")


if __name__ == "__main__":
    main()
