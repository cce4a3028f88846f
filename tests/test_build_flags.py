"""CPU: the device code is built without packed-fp32 VALU instructions
(csrc/Makefile NOPK; why: tests/test_gpu_coresidence.py).
Compiles the sources that used them most to gfx950 assembly with the Makefile's
own flags and checks that no v_pk_{fma,mul,add}_f32 is left."""
import os
import re
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "point-cloud-flow-matching_amd", "csrc")


def _makefile_flags():
    out = subprocess.run(["make", "-s", "-C", CSRC, "print-flags"], capture_output=True,
                         text=True, timeout=60, check=True).stdout.strip()
    return out.split()


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
@pytest.mark.parametrize("src", ["voxel.hip", "norm.hip", "chamfer.hip"])
def test_no_packed_fp32_in_device_code(tmp_path, src):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    flags = _makefile_flags()
    assert "-packed-fp32-ops" in flags
    out = tmp_path / (src + ".s")
    subprocess.run([hipcc, *flags, "--cuda-device-only", "-S", os.path.join(CSRC, src), "-o",
                    str(out)], check=True, capture_output=True, timeout=600)
    asm = out.read_text()
    assert "v_mfma" in asm or "v_fma" in asm  # real device code
    bad = re.findall(r"v_pk_(?:fma|mul|add)_f32", asm)
    assert not bad, f"{src}: {len(bad)} packed-fp32 instructions"
