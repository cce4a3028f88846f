"""Which kernel, running in ANOTHER process on the same GPU, corrupts the
devoxelization gather?  

tools/ddp_devox_probe.py showed that with two ranks sharing the GPU's CUs the
self-check (pcfm_debug_devox_verify, run right after each gather on the same
stream) finds outputs that were wrong when stored -- in 16-lane runs starting
at lane 48 -- and none when each rank has its own half of the CUs
(HSA_CU_MASK).  Inside one process kernels on one stream never overlap, so the
hazard is co-residence with a different kernel.  Here a victim process loops
the gather + self-check while an aggressor process loops one candidate kernel
for the same wall time; one JSON line per aggressor.

Usage (GPU box): python tools/coresidency_probe.py [seconds per aggressor]
                 python tools/coresidency_probe.py victim|aggressor NAME SECONDS"""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

AGGRESSORS = ["none", "devox", "conv_fwd", "conv_wgrad", "pointwise", "bn", "blas", "vox_bwd"]
SHAPES = [(8, 256, 4096, 16), (8, 256, 4096, 8), (8, 128, 4096, 32)]


def _canary(seconds):
    """A victim with no spills and no LDS: torch elementwise kernels whose
    result is compared with the first evaluation (bitwise)."""
    import torch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(8, 256, 4096, device=dev, generator=g)
    ref = torch.addcmul(x * 1.5 + 0.25, x, x)
    bad = torch.zeros((), dtype=torch.int64, device=dev)
    it = 0
    t0 = time.time()
    while time.time() - t0 < seconds:
        y = torch.addcmul(x * 1.5 + 0.25, x, x)
        bad += (y != ref).sum()
        it += 1
        if it % 50 == 0:
            torch.cuda.synchronize(dev)
    print(json.dumps({"iterations": it, "mismatches": int(bad), "calls": it,
                      "bad_weight_sums": 0, "records": []}), flush=True)


def _victim(seconds):
    import torch
    from pcfm import ops
    if os.environ.get("PROBE_VICTIM") == "canary":
        return _canary(seconds)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    if os.environ.get("PROBE_SAME_PROCESS"):
        # the aggressor in this process on a second stream (a Python thread)
        import threading
        side = torch.cuda.Stream(dev)

        def agg():
            with torch.cuda.stream(side):
                _aggressor(os.environ["PROBE_SAME_PROCESS"], seconds + 2, quiet=True)
        th = threading.Thread(target=agg, daemon=True)
        th.start()
    cases = []
    for b, c, n, r in SHAPES:
        coords = torch.rand(b, 3, n, device=dev, generator=g) * (r - 1)
        feat = torch.randn(b, c, r ** 3, device=dev, generator=g)
        scale = torch.rand(b, c, device=dev, generator=g)
        add = torch.randn(b, c, n, device=dev, generator=g)
        cases.append((r, coords, feat, scale, add))
    it = 0
    t0 = time.time()
    while time.time() - t0 < seconds:
        for r, coords, feat, scale, add in cases:
            ops.trilinear_devoxelize_scale_add(r, True, coords, feat, scale, add)
        it += 1
        if it % 50 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    if os.environ.get("PROBE_SAME_PROCESS"):
        th.join()  # the side stream's work drains before the process exits
        torch.cuda.synchronize(dev)
    rep = ops.devox_verify.report()
    rep["iterations"] = it
    print(json.dumps(rep), flush=True)


def _aggressor(name, seconds, quiet=False):
    import torch
    from pcfm import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    if name == "none":
        time.sleep(seconds)
        print(json.dumps({"iterations": 0}))
        return
    if name == "devox":
        b, c, n, r = SHAPES[0]
        coords = torch.rand(b, 3, n, device=dev, generator=g) * (r - 1)
        feat = torch.randn(b, c, r ** 3, device=dev, generator=g)
        add = torch.randn(b, c, n, device=dev, generator=g)
        scale = torch.rand(b, c, device=dev, generator=g)
        fn = lambda: ops.trilinear_devoxelize_scale_add(r, True, coords, feat, scale, add)  # noqa
    elif name in ("conv_fwd", "conv_wgrad"):
        b, c, r = 8, 256, 16
        x = torch.randn(b, c, r, r, r, device=dev, generator=g)
        w = torch.randn(c, c, 3, 3, 3, device=dev, generator=g) * 0.02
        xs = ops.conv3d_split(x)
        img = ops.conv3d_prep_weight(w, False)
        if name == "conv_fwd":
            fn = lambda: ops.conv3d_igemm_split(xs, img, None, b, c, c, r, "conv3d_fwd")  # noqa
        else:
            fn = lambda: ops.conv3d_wgrad_split(xs, xs, b, c, c, r)  # noqa
    elif name == "pointwise":
        x = torch.randn(8, 256, 20000, device=dev, generator=g)
        w = torch.randn(256, 256, device=dev, generator=g) * 0.05
        fn = lambda: ops.pointwise_forward(x, w, None)  # noqa
    elif name == "bn":
        x = torch.randn(8, 256, 20000, device=dev, generator=g)
        gm, bt = torch.ones(256, device=dev), torch.zeros(256, device=dev)
        rm, rv = torch.zeros(256, device=dev), torch.ones(256, device=dev)
        fn = lambda: ops.bn_act_forward(x, gm, bt, 1e-5, 0.0, 0.1, rm, rv, None)  # noqa
    elif name == "blas":
        a = torch.randn(4096, 4096, device=dev, generator=g).bfloat16()
        fn = lambda: a @ a  # noqa
    elif name == "vox_bwd":
        b, c, n, r = 8, 128, 20000, 32
        ind = torch.randint(0, r ** 3, (b, n), device=dev, dtype=torch.int32, generator=g)
        cnt = torch.ones(b, r ** 3, device=dev, dtype=torch.int32)
        gy = torch.randn(b, c, r ** 3, device=dev, generator=g)
        fn = lambda: ops.avg_voxelize_backward(gy, ind, cnt)  # noqa
    else:
        raise SystemExit(f"unknown aggressor {name}")
    it = 0
    t0 = time.time()
    while time.time() - t0 < seconds:
        fn()
        it += 1
        if it % 20 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    if not quiet:
        print(json.dumps({"iterations": it}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "victim":
        return _victim(float(sys.argv[2]))
    if len(sys.argv) > 1 and sys.argv[1] == "aggressor":
        return _aggressor(sys.argv[2], float(sys.argv[3]))
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 12.0
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else AGGRESSORS
    me = os.path.abspath(__file__)
    for spec in names:
        # NAME | NAME@canary (torch elementwise victim) | NAME@stream (same process)
        name, _, how = spec.partition("@")
        env = dict(os.environ, PCFM_DEVOX_VERIFY="1")
        if how == "canary":
            env["PROBE_VICTIM"] = "canary"
        agg_name = name
        if how == "stream":
            env["PROBE_SAME_PROCESS"] = name
            agg_name = "none"
        agg = subprocess.Popen([sys.executable, me, "aggressor", agg_name, str(secs + 4)],
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
        vic = subprocess.run([sys.executable, me, "victim", str(secs)], capture_output=True,
                             text=True, env=env, timeout=secs + 120)
        a_out, a_err = agg.communicate(timeout=secs + 120)
        res = {"aggressor": spec, "victim_rc": vic.returncode, "aggressor_rc": agg.returncode}
        try:
            res["victim"] = json.loads(vic.stdout.strip().splitlines()[-1])
            res["aggressor_iterations"] = json.loads(a_out.strip().splitlines()[-1])["iterations"]
        except (IndexError, ValueError, KeyError):
            res["victim_err"] = vic.stderr[-2000:]
            res["aggressor_err"] = a_err[-2000:]
        print(json.dumps(res), flush=True)
        if vic.returncode != 0 or agg.returncode != 0:
            sys.exit(1)


if __name__ == "__main__":
    main()
