"""Subprocess of tests/test_gpu_ops.py::test_chamfer_c2_product_path: the Chamfer
kernel the product runs at C2 (B=8, N=M=20000: 4e8 pairs per cloud pair, below
the 2^31 culling threshold -> the brute-force split-candidate search with its
64-bit atomicMin merge), with PCFM_CHAMFER_CULL_PAIRS unset (the GPU test
session sets it for the culled-path tests, and the library caches it).

Inputs carry exact hits and duplicate candidates (ties -> lowest index, the
reference's strict `<` scan, chamfer3D.cu:36-68, :126).  A sample of queries
per direction is checked bit-exactly against the oracle's full scan over the
whole candidate cloud; the backward (chamfer3D.cu:155-174) against the oracle
over the full clouds at 1e-5.  Writes a JSON report to argv[1]."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402


def main():
    assert "PCFM_CHAMFER_CULL_PAIRS" not in os.environ
    from pcfm import _lib, ops
    _lib.load()
    b, n = 8, 20000
    assert n * n < 2 ** 31  # the brute-force path (csrc/chamfer.hip use_cull)
    g = np.random.default_rng(20000)
    a = g.standard_normal((b, n, 3)).astype(np.float32)
    c = g.standard_normal((b, n, 3)).astype(np.float32)
    c[:, 5000:6000] = c[:, 1000:2000]     # duplicate candidates: ties inside xyz2
    a[:, :3000] = c[:, 4000:7000]         # queries on candidates, incl. the duplicates
    a[:, 19000:] = a[:, 18000:19000]      # duplicates inside xyz1 (ties for direction 2)
    dev = "cuda"
    x1, x2 = torch.from_numpy(a).to(dev), torch.from_numpy(c).to(dev)
    d1 = torch.empty(b, n, device=dev)
    d2 = torch.empty(b, n, device=dev)
    i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    i2 = torch.empty(b, n, dtype=torch.int32, device=dev)
    assert ops.chamfer_3D.forward(x1, x2, d1, d2, i1, i2) == 1
    d1, d2, i1, i2 = (t.cpu().numpy() for t in (d1, d2, i1, i2))
    # sampled queries: 300 per batch element and direction, incl. the tie blocks
    q = np.concatenate([g.choice(n, 200, replace=False), np.arange(4990, 5090),
                        np.arange(18950, 19050)])
    mism = {"d1": 0, "i1": 0, "d2": 0, "i2": 0}
    checked = 0
    for bb in range(b):
        e = O.chamfer_fwd(a[bb:bb + 1, q], c[bb:bb + 1])
        mism["d1"] += int(np.sum(d1[bb, q] != e[0][0]))
        mism["i1"] += int(np.sum(i1[bb, q] != e[2][0]))
        e = O.chamfer_fwd(c[bb:bb + 1, q], a[bb:bb + 1])
        mism["d2"] += int(np.sum(d2[bb, q] != e[0][0]))
        mism["i2"] += int(np.sum(i2[bb, q] != e[2][0]))
        checked += 2 * len(q)
    ties = int(np.sum(d1[:, :3000] == 0.0))
    # backward over the full clouds with the (checked) indices
    gd1 = g.random((b, n)).astype(np.float32)
    gd2 = g.random((b, n)).astype(np.float32)
    g1 = torch.zeros(b, n, 3, device=dev)
    g2 = torch.zeros(b, n, 3, device=dev)
    assert ops.chamfer_3D.backward(x1, x2, g1, g2, torch.from_numpy(gd1).to(dev),
                                   torch.from_numpy(gd2).to(dev),
                                   torch.from_numpy(i1).to(dev), torch.from_numpy(i2).to(dev)) == 1
    e1, e2 = O.chamfer_bwd(a, c, gd1, gd2, i1, i2)
    g1, g2 = g1.cpu().numpy(), g2.cpu().numpy()

    def rel(x, y):
        return float(np.max(np.abs(x - y) / (np.abs(y) + 1e-5)))

    json.dump({"mismatches": mism, "queries_checked": checked, "exact_hits": ties,
               "bwd_rel1": rel(g1, e1), "bwd_rel2": rel(g2, e2),
               "bwd_close": bool(np.allclose(g1, e1, rtol=1e-5, atol=1e-5)
                                 and np.allclose(g2, e2, rtol=1e-5, atol=1e-5))},
              open(sys.argv[1], "w"))


if __name__ == "__main__":
    main()
