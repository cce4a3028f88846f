"""Diagnosis of the devoxelization results that differed between identical runs
when two ranks shared one GPU: runs the two-rank helper
tests/helpers/ddp_grad_rank.py (ranks concurrent) with the in-stream self-check
(PCFM_DEVOX_VERIFY=1: every devoxelization output recomputed in the plainest
form right after the gather and compared bit for bit) and the op-level trace,
once per variant, and prints one JSON line per run:

  shared    both ranks on all 256 CUs
  cu_split  rank 0 on CUs 0-127, rank 1 on CUs 128-255 (HSA_CU_MASK)

Usage (GPU box): python tools/ddp_devox_probe.py [runs per variant]"""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPER = os.path.join(REPO, "tests", "helpers", "ddp_grad_rank.py")


def run(variant, k, port):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PCFM_DEVOX_VERIFY="1",
               PCFM_DDP_TRACE="1")
    if variant == "cu_split":
        env["PCFM_DDP_CU_SPLIT"] = "1"
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "grad.json")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(port), HELPER, out]
        p = subprocess.run(cmd, timeout=300, env=env, cwd=REPO, capture_output=True, text=True)
        res = {"variant": variant, "run": k, "rc": p.returncode}
        if p.returncode != 0:
            res["stderr_tail"] = p.stderr[-3000:]
            return res
        ranks = [json.load(open(f"{out}.{r}")) for r in range(2)]
    for d_ in ranks:
        tr = d_.get("trace") or {}
        res[f"rank{d_['rank']}"] = {
            "max_rel": d_["max_rel"], "differ": d_["differ"], "unreproducible": d_["unreproducible"],
            "losses_equal_ref": d_["losses"] == d_["ref_losses"][d_["rank"]],
            "first_diff_ddp_vs_ref": tr.get("ddp_vs_ref"),
            "first_diff_ref_vs_again": tr.get("ref_vs_again"),
            "devox_elements": tr.get("devox"), "devox_verify": d_.get("devox_verify"),
            "cu_mask": d_.get("cu_mask")}
    return res


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    port = 29600
    for variant in ("shared", "cu_split"):
        for k in range(n):
            port += 1
            res = run(variant, k, port)
            print(json.dumps(res), flush=True)
            if res["rc"] != 0:  # a crashed run ends the probe (no retries)
                sys.exit(1)


if __name__ == "__main__":
    main()
