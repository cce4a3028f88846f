"""EMD forward at the bench size (B=8, N=M=2048): wall ms per call (events
and host clock) for the default form and PCFM_EMD_FORM=split, one JSON line
each.  Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402


def main():
    from pcfm import _lib
    from PyTorchEMD.emd import earth_mover_distance
    _lib.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    b, n = 8, int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    p1 = torch.rand(b, n, 3, device=dev, generator=g)
    p2 = torch.rand(b, n, 3, device=dev, generator=g)
    for form in ("rowpass", "split"):
        os.environ["PCFM_EMD_FORM"] = form
        x = p1.detach().requires_grad_(True)  # the forward a backward follows: match kept
        for _ in range(3):
            earth_mover_distance(x, p2, transpose=False)
        torch.cuda.synchronize(dev)
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(reps):
            d = earth_mover_distance(x, p2, transpose=False)
        e1.record()
        torch.cuda.synchronize(dev)
        host = (time.perf_counter() - t0) * 1e3 / reps
        print(json.dumps({"form": form, "b": b, "n": n, "fwd_ms_events": e0.elapsed_time(e1) / reps,
                          "fwd_ms_host": host, "cost0": float(d[0])}), flush=True)


if __name__ == "__main__":
    main()
