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


_LLVM = "/opt/rocm/lib/llvm/bin"
_LIB = os.path.join(CSRC, "libpcfm_hip.so")


@pytest.mark.skipif(not (os.path.exists(os.path.join(_LLVM, "clang-offload-bundler"))
                         and os.path.exists(_LIB)), reason="no built library / llvm tools")
def test_shipped_library_has_no_packed_fp32(tmp_path):
    """The built libpcfm_hip.so itself (not a fresh compile): every gfx950 code
    object in its fat binary -- one offload bundle per source -- disassembled,
    no v_pk_{fma,mul,add}_f32 (a stale object built before the NOPK flag would
    still carry them; the Makefile's build/.flags stamp rebuilds on a flag change)."""
    fb = tmp_path / "fatbin.bin"
    subprocess.run([os.path.join(_LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}",
                    _LIB, str(tmp_path / "lib.so")], check=True, capture_output=True, timeout=120)
    data = fb.read_bytes()
    starts = [m.start() for m in re.finditer(rb"__CLANG_OFFLOAD_BUNDLE__", data)]
    assert len(starts) >= 10  # one bundle per source file of the Makefile
    n_mfma = 0
    for k, s in enumerate(starts):
        part = tmp_path / f"b{k}.bin"
        part.write_bytes(data[s: starts[k + 1] if k + 1 < len(starts) else len(data)])
        co = tmp_path / f"b{k}.o"
        subprocess.run([os.path.join(_LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}",
                        f"--output={co}"], check=True, capture_output=True, timeout=120)
        asm = subprocess.run([os.path.join(_LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", str(co)],
                             check=True, capture_output=True, text=True, timeout=300).stdout
        bad = re.findall(r"v_pk_(?:fma|mul|add)_f32", asm)
        assert not bad, f"bundle {k}: {len(bad)} packed-fp32 instructions"
        n_mfma += asm.count("v_mfma")
    assert n_mfma > 0  # the disassembly is real device code
