"""Per-step kernel breakdown of a bench.py rocprofv3 trace: steps are delimited
by the optimizer's fused Adam kernels; the last K steps are averaged.  Dev tool."""
import collections
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from kstats import load, short  # noqa: E402

path, k = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = load(path)
idx = [i for i, (n, _) in enumerate(rows) if "adam" in n.lower()]
ends, prev = [], None
for i in idx:
    if prev is not None and i - prev > 50:
        ends.append(prev)
    prev = i
ends.append(prev)
lo, hi = ends[-k - 1] + 1, ends[-1] + 1
sel = rows[lo:hi]
agg = collections.defaultdict(lambda: [0, 0.0])
for n, d in sel:
    s = short(n)
    agg[s][0] += 1
    agg[s][1] += d
tot = sum(v[1] for v in agg.values())
print(f"{k} steps, {len(sel)} kernels, kernel time {tot / 1000 / k:.2f} ms/step")
for s, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{s[:80]:80s} {c / k:6.1f}/step {t / 1000 / k:8.3f} ms/step {100 * t / tot:5.1f}%")
