"""Dev probe: how the LDS-DMA voxel-conv kernel's time scales with the work its
occupancy masks leave (synthetic masks), and with the batch (rounds of blocks).
Prints one JSON line per case: {case, ms}.  Usage (GPU box):
    python tools/conv_occ_probe.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402

from pcfm import _lib, ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    _lib.load()
    c, r = 128, 32
    V = r ** 3
    for b in (2, 4, 8):
        x = torch.randn(b, c, r, r, r, device="cuda")
        xs = ops.conv3d_split(x)
        w = torch.randn(c, c, 3, 3, 3, device="cuda") * 0.05
        img = ops.conv3d_prep_weight(w, False)
        bias = torch.zeros(c, device="cuda")
        nt = V // 256
        full = (1 << 27) - 1

        def masks(tile_fn):
            m = torch.zeros(b * (nt + V // 64), dtype=torch.int64)
            for bb in range(b):
                for t in range(nt):
                    m[bb * nt + t] = tile_fn(bb, t)
            m = torch.where(m >= 2 ** 31, m - 2 ** 32, m).to(torch.int32)
            return m.cuda()

        cases = {
            "none": None,
            "all": masks(lambda bb, t: full | (1 << 31)),
            "half_first_tiles": masks(lambda bb, t: (full | (1 << 31)) if t < nt // 2 else 0),
            "half_alt_tiles": masks(lambda bb, t: (full | (1 << 31)) if t % 2 == 0 else 0),
            "quarter_tiles": masks(lambda bb, t: (full | (1 << 31)) if t % 4 == 0 else 0),
            "taps_9_of_27": masks(lambda bb, t: (1 << 9) - 1),
            "taps_18_of_27": masks(lambda bb, t: (1 << 18) - 1),
        }
        for name, m in cases.items():
            for mode in ((1, 2) if m is not None else (0,)):
                if name.startswith("taps") and mode == 2:
                    continue
                ms = timeit(lambda: ops.conv3d_igemm_split(xs, img, bias, b, c, c, r, "x", occ=m,
                                                           occ_mode=mode))
                print(json.dumps({"b": b, "case": name, "mode": mode, "ms": ms}), flush=True)


if __name__ == "__main__":
    main()
