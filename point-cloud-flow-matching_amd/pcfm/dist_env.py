"""Environment of the RCCL process group, set before `init_process_group`.

The reference's one exchange step is DDP's gradient all-reduce
(/root/reference/train.py:240-244, util.py:71-84).  torch's DDP reducer issues
it as an fp32 SUM: with no communication hook installed it runs
`c10d::_AllReduceBySumCommHook` (torch/csrc/distributed/c10d/
default_comm_hooks.hpp), the division by the world size fused into the copy
into the bucket (`torch::distributed::reducer::mul_out`), so the reduce op is
SUM -- not AVG or PREMUL_SUM.

Which RCCL device function performs that SUM depends on the algorithm RCCL
picks per call.  In the gfx950 code object of the librccl.so torch ships, the
ring kernels `runRing<float, FuncSum, {Simple, LL, LL128}>` carry no packed
fp32 VALU instruction, but `runTreeUpDown<float, FuncSum, Simple>` and every
`FuncPreMulSum` float kernel do (v_pk_add_f32 / v_pk_mul_f32).  Packed-fp32
results in lanes 48-63 were measured wrong on MI355X while MFMA-heavy waves of
another kernel share the SIMD, and under DDP the
all-reduce runs on RCCL's stream concurrently with this library's MFMA
backward.  So the algorithm is pinned to Ring; tests/test_codeobj.py checks
the code object and turns red if an RCCL update adds packed fp32 to the ring
kernels.  Ring is also what RCCL picks for the large buckets (25 MB) of this
all-reduce on one xGMI node; the small-message LL / tree choices it gives up
cost nothing measurable at four buckets per step."""
from __future__ import annotations

import os
import sys

RCCL_ALGO = "Ring"


def pin_rccl_env(environ=None) -> dict:
    """Set NCCL_ALGO=Ring in `environ` (default os.environ) unless the caller
    has set PCFM_KEEP_NCCL_ALGO=1 to keep a different choice; returns the
    settings in force.  Must run before the process group is created (RCCL
    reads it at communicator init) -- and, for ranks started by a launcher,
    in the launcher's environment too."""
    env = os.environ if environ is None else environ
    cur = env.get("NCCL_ALGO")
    if cur and cur != RCCL_ALGO and env.get("PCFM_KEEP_NCCL_ALGO") == "1":
        print(f"[pcfm] NCCL_ALGO={cur} kept (PCFM_KEEP_NCCL_ALGO=1): the RCCL kernels it "
              "selects are not checked for packed fp32 (pcfm/dist_env.py)", file=sys.stderr)
    else:
        env["NCCL_ALGO"] = RCCL_ALGO
    return {"NCCL_ALGO": env["NCCL_ALGO"]}
