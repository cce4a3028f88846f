"""A/B timing of the head weight gradient rows_wgrad_bf16 at the C2 train-step
shapes (dev tool): PCFM_LIB=<variant> PCFM_RW_BPC=<blocks per CU> python
tools/rows_ab.py tag.  JSON line; also the max relative difference against an
fp64 reference of the same product."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402
from tools.scatter_ab import timeit  # noqa: E402


def main():
    res = {"tag": sys.argv[1] if len(sys.argv) > 1 else "main",
           "bpc": os.environ.get("PCFM_RW_BPC", "2")}
    g = torch.Generator(device="cuda").manual_seed(0)
    for rows, m, n in ((160000, 512, 512), (160000, 512, 384), (160000, 6, 512)):
        a = torch.randn(rows, m, device="cuda", generator=g).bfloat16()
        b = torch.randn(rows, n, device="cuda", generator=g).bfloat16()
        t = timeit(lambda: ops.rows_wgrad_bf16(a, b))
        ref = a.double().t() @ b.double()
        err = float(((ops.rows_wgrad_bf16(a, b).double() - ref).abs().max() / ref.abs().max()))
        res[f"R{rows}M{m}N{n}"] = {"ms": t, "rel_err": err}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
