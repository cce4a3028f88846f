"""The hipBLASLt kernel torch runs for the co-residence probe's "blas" aggressor
(tools/coresidency_probe.py: bf16 4096 x 4096 @ 4096 x 4096): run it under
`rocprofv3 --kernel-trace --stats` to name the kernel, whose resource metadata
tools/co_resources.py then reads from the library's code object."""
import torch

g = torch.Generator(device="cuda").manual_seed(0)
a = torch.randn(4096, 4096, device="cuda", generator=g).bfloat16()
b = torch.randn(4096, 4096, device="cuda", generator=g).bfloat16()
for _ in range(5):
    c = a @ b
torch.cuda.synchronize()
print(float(c.float().abs().mean()))
