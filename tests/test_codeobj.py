"""CPU: what the shipped device code contains (tests/helpers/codeobj.py).

* The built libpcfm_hip.so -- the file the GPU runs load, not a fresh compile --
  carries no packed-fp32 VALU instruction in any kernel (csrc/Makefile NOPK;
  DESIGN.md section 6).
* The RCCL device functions the DDP gradient all-reduce is pinned to
  (NCCL_ALGO=Ring, pcfm/dist_env.py: fp32 SUM, ring, any protocol) carry none
  in the gfx950 code object of the librccl.so torch loads; neither does the
  generic kernel that dispatches to them, nor the MSCCL fp32-sum kernels.  If an
  RCCL update changes that, this turns red.
* The pin is set by both launch paths before the process group exists."""
import os
import re
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(HERE, "helpers"))
import codeobj  # noqa: E402

LIB = os.path.join(REPO, "point-cloud-flow-matching_amd", "csrc", "libpcfm_hip.so")
needs_tools = pytest.mark.skipif(not codeobj.available(), reason="ROCm LLVM tools absent")


@needs_tools
@pytest.mark.skipif(not os.path.exists(LIB), reason="libpcfm_hip.so not built")
def test_shipped_library_has_no_packed_fp32(tmp_path):
    cos = codeobj.extract(LIB, str(tmp_path))
    assert cos, "no gfx950 code object in libpcfm_hip.so"
    kernels, bad = 0, {}
    for co in cos:
        kernels += len(codeobj.kernel_resources(co))
        for fn, n in codeobj.count_per_function(co, []).items():
            if n:
                bad[fn] = n
    assert kernels > 100  # the whole library was read
    assert not bad, f"packed fp32 in the shipped library: {bad}"


@needs_tools
@pytest.mark.skipif(not os.path.exists(LIB), reason="libpcfm_hip.so not built")
def test_weight_gradient_claims_its_cus(tmp_path):
    """conv3_wgrad3 (768 threads = 3 waves per SIMD, LDS-DMA) allocates 168 VGPRs
    per lane, 504 of each SIMD's 512: no wave of another kernel needing more than
    8 can share a CU with it (PCFM_CLAIM_VGPRS)."""
    found = 0
    for co in codeobj.extract(LIB, str(tmp_path)):
        res = codeobj.kernel_resources(co)
        for k, v in res.items():
            if "conv3_wgrad3_kernel" in k:
                regs = codeobj.descriptor_registers(co, k)
                assert v["wg"] == 768 and regs["alloc"] == 168, (k, v, regs)
                assert v["scratch"] == 0
                found += 1
    assert found == 1


def _librccl():
    import torch
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else None


@needs_tools
@pytest.mark.skipif(_librccl() is None, reason="torch ships no librccl.so")
def test_rccl_ring_fp32_sum_kernels_have_no_packed_fp32(tmp_path):
    cos = codeobj.extract(_librccl(), str(tmp_path))
    assert len(cos) == 1
    co = cos[0]
    fns = codeobj.functions(co)
    ring = [f for f in fns if re.search(r"runRingIf7FuncSumIfE", f)]
    generic = [f for f in fns if "rcclGenericKernel" in f]
    msccl = [f for f in fns if re.search(r"mscclKernel_Sum_float_", f)]
    # Simple (several slice shapes), LL and LL128, each unrolled 1 / 2 / 4
    assert len(ring) >= 9 and generic, (len(ring), len(generic))
    counts = codeobj.count_per_function(co, ring + generic + msccl)
    bad = {f: n for f, n in counts.items() if n}
    assert not bad, f"packed fp32 in the pinned RCCL kernels: {bad}"
    # the kernels the pin avoids: documents why it exists (not asserted -- an
    # RCCL that cleans them up only makes the pin unnecessary)
    tree = [f for f in fns if re.search(r"runTreeUpDownIf7FuncSumIfE", f)]
    avoided = sum(codeobj.count_per_function(co, tree).values()) if tree else 0
    print(f"ring fp32-sum functions: {len(ring)} clean; tree up/down: {avoided} packed fp32")


def test_pin_sets_ring(monkeypatch):
    from pcfm.dist_env import pin_rccl_env
    env = {}
    assert pin_rccl_env(env) == {"NCCL_ALGO": "Ring"} and env["NCCL_ALGO"] == "Ring"
    env = {"NCCL_ALGO": "Tree"}
    pin_rccl_env(env)
    assert env["NCCL_ALGO"] == "Ring"  # overridden unless explicitly kept
    env = {"NCCL_ALGO": "Tree", "PCFM_KEEP_NCCL_ALGO": "1"}
    pin_rccl_env(env)
    assert env["NCCL_ALGO"] == "Tree"


def test_launch_paths_pin_before_init(monkeypatch):
    """pcfm.train.init_distributed pins for the RCCL backend before creating the
    group; bench.py's launcher passes the pin to its ranks and each rank pins
    again before init (the driver starts ranks with torch.distributed.run)."""
    import torch
    import torch.distributed as dist
    from pcfm import train as T

    calls = []
    monkeypatch.delenv("NCCL_ALGO", raising=False)
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setattr(torch.cuda, "set_device", lambda *a: None)
    monkeypatch.setattr(dist, "is_initialized", lambda: False)
    monkeypatch.setattr(dist, "init_process_group",
                        lambda **kw: calls.append((kw["backend"], os.environ.get("NCCL_ALGO"))))
    T.init_distributed("nccl")
    assert calls == [("nccl", "Ring")]
    src = open(os.path.join(REPO, "bench.py")).read()
    launcher = src[src.index("def launch_ranks"):src.index("def main")]
    assert "pin_rccl_env(env)" in launcher and "subprocess.call(cmd, env=env)" in launcher
    main = src[src.index("def main"):]
    assert main.index("pin_rccl_env()") < main.index("dist.init_process_group")
