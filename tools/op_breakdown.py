"""Per-launch kernel composition of the segment-sum ops in a bench.py kernel
trace: finds each `seg_units<TAPS>` dispatch, takes the seg_sort before it and
the transpose / unit_gather / part_sum after it, and averages over the last K
steps.  TAPS=8 is trilinear_devoxelize_bwd, TAPS=1 avg_voxelize_fwd (with its
vox_ind kernel).  Dev tool."""
import collections
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from kstats import load, short  # noqa: E402

rows = [(short(n).replace("void ", ""), d) for n, d in load(sys.argv[1])]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
groups = collections.defaultdict(list)
for i, (n, d) in enumerate(rows):
    if "seg_units_kernel" not in n:
        continue
    taps = n.split("<")[1].rstrip(">")
    comp = {}
    j = i - 1
    while j >= 0 and "seg_sort_kernel" not in rows[j][0]:
        j -= 1
    comp["seg_sort_kernel"] = rows[j][1]
    if taps == "1" and j > 0 and "vox_ind_kernel" in rows[j - 1][0]:
        comp["vox_ind_kernel"] = rows[j - 1][1]
    comp[n.split("::")[-1]] = d
    for k in range(i + 1, min(i + 6, len(rows))):
        nk = rows[k][0].split("::")[-1]
        if nk.startswith(("seg_transpose", "seg_unit_gather", "seg_part_sum")):
            comp[nk] = rows[k][1]
        if nk.startswith("seg_part_sum"):
            break
    groups[taps].append(comp)
names = {"8": "trilinear_devoxelize_bwd", "1": "avg_voxelize_fwd"}
for taps, comps in groups.items():
    comps = comps[-6 * steps:]  # 6 launches per step
    keys = list(comps[-1].keys())
    avg = {k: sum(c.get(k, 0.0) for c in comps) / len(comps) for k in keys}
    print(f"{names.get(taps, taps)}: {len(comps)} launches, kernel time per launch "
          f"{sum(avg.values()):.1f} us")
    for k, v in avg.items():
        print(f"    {k:40s} {v:8.1f} us")
