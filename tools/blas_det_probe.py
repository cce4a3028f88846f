"""Dev probe: bitwise reproducibility of the library GEMMs (torch -> hipBLASLt /
rocBLAS) at the model's shapes over repeated calls; run two copies at once to
put the GPU under contention.  Prints {case, mismatching_calls}."""
import json
import os
import sys

import torch
import torch.nn.functional as F


def main():
    reps = int(os.environ.get("REPS", "40"))
    g = torch.Generator(device="cuda").manual_seed(0)
    cases = []
    # SE3d MLP (fp32, autocast off): (B, C) x (C/8, C)^T, then (B, C/8) x (C, C/8)^T
    for c in (128, 256):
        m = torch.randn(8, c, device="cuda", generator=g)
        w1 = torch.randn(c // 8, c, device="cuda", generator=g)
        w2 = torch.randn(c, c // 8, device="cuda", generator=g)
        cases.append((f"se_mlp_c{c}",
                      lambda m=m, w1=w1, w2=w2: torch.sigmoid(F.linear(F.relu(F.linear(m, w1)), w2))))
    # per-cloud fp32 Linears (embeddings, FiLM affines, global MLP)
    for k, n in ((256, 256), (256, 512), (256, 1024)):
        a = torch.randn(8, k, device="cuda", generator=g)
        w = torch.randn(n, k, device="cuda", generator=g)
        b = torch.randn(n, device="cuda", generator=g)
        cases.append((f"linear_8x{k}x{n}", lambda a=a, w=w, b=b: F.linear(a, w, b)))
    # the head trunk's bf16 GEMMs (B*N = 160000 rows)
    for k, n in ((326, 512), (512, 512), (512, 6)):
        a = torch.randn(160000, k, device="cuda", generator=g).bfloat16()
        w = torch.randn(n, k, device="cuda", generator=g).bfloat16()
        cases.append((f"bf16_160000x{k}x{n}", lambda a=a, w=w: F.linear(a, w)))
        gy = torch.randn(160000, n, device="cuda", generator=g).bfloat16()
        cases.append((f"bf16_dgrad_160000x{n}x{k}", lambda gy=gy, w=w: gy @ w))
    for name, fn in cases:
        ref = fn().clone()
        bad = 0
        for _ in range(reps):
            if not torch.equal(fn(), ref):
                bad += 1
        torch.cuda.synchronize()
        print(json.dumps({"case": name, "mismatching_calls": bad, "of": reps}), flush=True)


if __name__ == "__main__":
    main()
