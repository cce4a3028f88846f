"""Per-kernel averages of rocprofv3 --pmc counter CSVs (dev tool):
python tools/pmc_sum.py <dir> [<dir> ...] [--match REGEX]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    pat = None
    if "--match" in args:
        i = args.index("--match")
        pat = args[i + 1]
        args = args[:i] + args[i + 2:]
    agg = defaultdict(lambda: defaultdict(list))
    for d in args:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))
                if pat and not re.search(pat, n):
                    continue
                agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, cs in agg.items():
        print(n[:80])
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
