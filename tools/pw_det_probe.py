"""Dev probe: bitwise reproducibility of the pointwise weight gradient
(pcfm_pointwise_wgrad) over repeated calls, at ContextNet head_out's shape
(cin 256, cout 64) and others.  Prints one JSON line per shape."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402

from pcfm import _lib, ops  # noqa: E402

_lib.load()
for b, cin, cout, n in ((8, 256, 64, 4096), (8, 256, 64, 20000), (8, 128, 128, 4096),
                        (8, 896, 256, 4096)):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(b, cin, n, device="cuda", generator=g)
    dy = torch.randn(b, cout, n, device="cuda", generator=g)
    ref = ops.pointwise_backward_weight(x, dy)
    bad = 0
    for _ in range(50):
        junk = torch.randn(64 << 20, device="cuda")  # churn the allocator / caches
        del junk
        if not torch.equal(ops.pointwise_backward_weight(x, dy), ref):
            bad += 1
    print(json.dumps({"shape": [b, cin, cout, n], "mismatching_calls_of_50": bad}), flush=True)
