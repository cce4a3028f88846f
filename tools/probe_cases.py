"""Median time per kernel for each case of tools/voxel_probe.py (6 cases in order)."""
import collections
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from kstats import load, short  # noqa: E402

rows = [(short(n), d) for n, d in load(sys.argv[1])]
rows = [r for r in rows if "pcfm" in r[0]]
per = len(rows) // 6
for ci, name in enumerate(["uR32", "uR16", "uR8", "nR32", "nR16", "nR8"]):
    agg = collections.defaultdict(list)
    for k, d in rows[ci * per:(ci + 1) * per]:
        agg[k.split("::")[-1]].append(d)
    print(name, {k: round(sorted(v)[len(v) // 2], 1) for k, v in agg.items()})
