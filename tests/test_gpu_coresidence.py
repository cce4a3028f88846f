"""GPU: kernels of this library sharing CUs with other kernels.

Measured on MI355X in round 4 (tools/coresidency_probe.py):
code using the packed-fp32 VALU instructions (v_pk_mul_f32 / v_pk_fma_f32 /
v_pk_add_f32, which hipcc emits for gfx950 from plain float code) returned wrong
values in lanes 48-63 of a wave while MFMA-heavy waves of another kernel ran on
the same CU -- the devoxelization gather beside the pointwise GEMM or the voxel
conv weight gradient: ~10^8 mismatching outputs in 12 s, whether the other
kernel came from a second process or from a second stream of the same process,
and none with the two kernels on disjoint CU halves (HSA_CU_MASK).  The library
is built without packed fp32 (csrc/Makefile NOPK); these tests run the gather
with its in-stream self-check (pcfm_debug_devox_verify) while a second stream
keeps MFMA kernels on the same CUs."""
import threading
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


# The conv_wgrad aggressor: passed on every full-suite run through round 5's
# end-of-round run, then from that afternoon on left the GPU with a memory-access
# fault in 4 of 4 runs (one in round 6), within seconds, after the pointwise
# variant in the same process; the same workload alone ran clean for 10 s. Since
# round 6 conv3_wgrad3 claims its CU's whole register file, so only kernels of
# <= 8 VGPRs could share a CU with it; that fix has not
# been run here (re-running a workload known to fault the shared pool was not
# allowed), so this variant still runs only on request.
_STRESS = __import__("os").environ.get("PCFM_CORESIDENCE_STRESS") == "1"


@pytest.mark.parametrize("aggressor", [
    "pointwise",
    pytest.param("conv_wgrad", marks=pytest.mark.skipif(
        not _STRESS, reason="faults the GPU on this pool since round 5 (PCFM_CORESIDENCE_STRESS=1 runs it)"))])
def test_devox_gather_exact_beside_mfma_kernels(aggressor, report):
    from pcfm import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    cases = []
    for b, c, n, r in ((8, 256, 4096, 16), (8, 256, 4096, 8), (8, 128, 4096, 32)):
        cases.append((r, torch.rand(b, 3, n, device=dev, generator=g) * (r - 1),
                      torch.randn(b, c, r ** 3, device=dev, generator=g),
                      torch.rand(b, c, device=dev, generator=g),
                      torch.randn(b, c, n, device=dev, generator=g)))
    if aggressor == "pointwise":
        x = torch.randn(8, 256, 20000, device=dev, generator=g)
        w = torch.randn(256, 256, device=dev, generator=g) * 0.05
        fn = lambda: ops.pointwise_forward(x, w, None)  # noqa: E731
    else:
        bsz, c, r = 8, 256, 16
        xs = ops.conv3d_split(torch.randn(bsz, c, r, r, r, device=dev, generator=g))
        fn = lambda: ops.conv3d_wgrad_split(xs, xs, bsz, c, c, r)  # noqa: E731
    torch.cuda.synchronize(dev)
    side = torch.cuda.Stream(dev)
    stop = threading.Event()
    launched = [0]

    def run_side():
        with torch.cuda.stream(side):
            while not stop.is_set():
                fn()
                launched[0] += 1
                if launched[0] % 20 == 0:
                    side.synchronize()
        side.synchronize()

    verify = ops.devox_verify
    old = verify.enabled
    verify.enabled, verify.rec, verify.calls = True, None, 0
    th = threading.Thread(target=run_side, daemon=True)
    th.start()
    try:
        t0, it = time.time(), 0
        while time.time() - t0 < 4.0:
            for r, coords, feat, scale, add in cases:
                ops.trilinear_devoxelize_scale_add(r, True, coords, feat, scale, add)
            it += 1
            if it % 50 == 0:
                torch.cuda.synchronize(dev)
    finally:
        stop.set()
        th.join()
        torch.cuda.synchronize(dev)
        rep = verify.report()
        verify.enabled = old
    rep["iterations"], rep["aggressor_launches"] = it, launched[0]
    report(f"coresidence_{aggressor}", rep)
    assert launched[0] > 0 and rep["calls"] > 0
    assert rep["mismatches"] == 0 and rep["bad_weight_sums"] == 0, rep
