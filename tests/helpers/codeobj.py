"""gfx950 code objects out of HIP fat binaries, their kernels' resource metadata
and per-function instruction counts (CPU only; ROCm's LLVM tools).

Used by tests/test_codeobj.py (the shipped libpcfm_hip.so carries no packed-fp32
VALU instructions; the RCCL kernels the gradient all-reduce is pinned to carry
none either) and by tools/co_resources.py (LDS, VGPR and
occupancy of the kernels the co-residence probe ran).

A `.so` built by hipcc keeps its device code in the `.hip_fatbin` section: one
clang offload bundle per translation unit (`__CLANG_OFFLOAD_BUNDLE__`), or one
compressed bundle (`CCOB`, torch's librccl.so).  `clang-offload-bundler` unpacks
both; `llvm-readelf --notes` prints the AMDGPU metadata (`amdhsa.kernels`)."""
from __future__ import annotations

import os
import re
import subprocess
from typing import Dict, Iterable, List

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
PACKED_F32 = re.compile(r"\bv_pk_(?:fma|mul|add)_f32\b")
_BUNDLE = b"__CLANG_OFFLOAD_BUNDLE__"


def tool(name: str) -> str:
    return os.path.join(LLVM, name)


def available() -> bool:
    return all(os.path.exists(tool(t)) for t in
               ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf", "llvm-objdump"))


def extract(path: str, workdir: str) -> List[str]:
    """The gfx950 code objects of `path` (a host .so with a .hip_fatbin section,
    or an ELF code object itself), written under `workdir`; their paths."""
    with open(path, "rb") as f:
        head = f.read(64)
    fat = os.path.join(workdir, os.path.basename(path) + ".fatbin")
    if head[:4] == b"\x7fELF" and b"amdgpu" not in _e_machine_str(path):
        subprocess.run([tool("llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", path,
                        os.devnull], check=True, capture_output=True, timeout=300)
    elif head[:4] == b"CCOB" or head.startswith(_BUNDLE):
        import shutil
        shutil.copyfile(path, fat)  # a bare (compressed) bundle, e.g. hipBLASLt's .co files
    else:
        return [path]  # already a device code object (.co / .hsaco)
    with open(fat, "rb") as f:
        data = f.read()
    starts = []
    if data[:4] == b"CCOB":
        starts = [0]  # one compressed bundle for the whole library
    else:
        i = data.find(_BUNDLE)
        while i != -1:
            starts.append(i)
            i = data.find(_BUNDLE, i + 1)
    ends = starts[1:] + [len(data)]
    out = []
    for k, (s, e) in enumerate(zip(starts, ends)):
        part = fat if (s, e) == (0, len(data)) else os.path.join(workdir, f"bundle{k}.bin")
        if part != fat:
            with open(part, "wb") as f:
                f.write(data[s:e])
        co = os.path.join(workdir, f"gfx950_{k}.co")
        r = subprocess.run([tool("clang-offload-bundler"), "--unbundle", "--type=o",
                            f"--input={part}", f"--targets={TARGET}", f"--output={co}"],
                           capture_output=True, timeout=600)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
        if part != fat:
            os.remove(part)
    os.remove(fat)
    return out


def _e_machine_str(path: str) -> bytes:
    r = subprocess.run([tool("llvm-readelf"), "-h", path], capture_output=True, timeout=60)
    return r.stdout.lower()


def functions(co: str) -> List[str]:
    """Names of the FUNC symbols of a code object (kernels and device functions)."""
    r = subprocess.run([tool("llvm-readelf"), "-s", "--wide", co], capture_output=True,
                       text=True, timeout=300, check=True)
    names = []
    for line in r.stdout.splitlines():
        f = line.split()
        if len(f) >= 8 and f[3] == "FUNC":
            names.append(f[7])
    return sorted(set(names))


def disassemble(co: str, symbols: Iterable[str] = ()) -> str:
    cmd = [tool("llvm-objdump"), "-d", co]
    syms = list(symbols)
    if syms:
        cmd.insert(2, "--disassemble-symbols=" + ",".join(syms))
    return subprocess.run(cmd, capture_output=True, text=True, timeout=900, check=True).stdout


def count_per_function(co: str, symbols: Iterable[str], pattern=PACKED_F32) -> Dict[str, int]:
    """{symbol: number of instructions matching `pattern` in its body}."""
    text = disassemble(co, symbols)
    counts: Dict[str, int] = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            counts.setdefault(cur, 0)
        elif cur is not None and pattern.search(line):
            counts[cur] += 1
    return counts


def kernel_resources(co: str) -> Dict[str, Dict[str, int]]:
    """{kernel name: {lds, vgpr, agpr, sgpr, wg, scratch}} from the AMDGPU
    metadata note.  `lds` is the static group segment: dynamic LDS (set at
    launch) comes on top."""
    r = subprocess.run([tool("llvm-readelf"), "--notes", co], capture_output=True, text=True,
                       timeout=300, check=True)
    keys = {".group_segment_fixed_size": "lds", ".vgpr_count": "vgpr", ".agpr_count": "agpr",
            ".sgpr_count": "sgpr", ".max_flat_workgroup_size": "wg",
            ".private_segment_fixed_size": "scratch", ".name": "name"}
    out: Dict[str, Dict[str, int]] = {}
    cur: Dict[str, object] = {}
    in_kernels = False

    def flush():
        if "name" in cur:
            name = str(cur.pop("name"))
            out[name] = {k: int(v) for k, v in cur.items()}

    for line in r.stdout.splitlines():
        if line.startswith("amdhsa.kernels:"):
            in_kernels = True
            continue
        if in_kernels and re.match(r"^amdhsa\.\w", line):
            in_kernels = False
        if not in_kernels:
            continue
        m = re.match(r"^  - (\.\w+):\s*(\S*)", line)  # a new kernel record
        if m:
            flush()
            cur = {}
        m = re.match(r"^\s{2,4}-?\s*(\.\w+):\s+(\S+)$", line)
        if m and m.group(1) in keys and line.startswith(("  - .", "    .")):
            cur[keys[m.group(1)]] = m.group(2)
    flush()
    return out


def descriptor_registers(co: str, kernel: str) -> Dict[str, int]:
    """Registers the hardware allocates per lane, from the kernel descriptor
    (`<kernel>.kd`): compute_pgm_rsrc1 bits 0-5 = total VGPR+AGPR granules of 8
    (gfx90a+ unified file), compute_pgm_rsrc3 bits 0-5 = ACCUM_OFFSET / 4 - 1.
    Hand-assembled kernels (Tensile) report only arch VGPRs in the metadata."""
    import struct
    r = subprocess.run([tool("llvm-readelf"), "-S", "-s", "--wide", co], capture_output=True,
                       text=True, timeout=300, check=True).stdout
    secs = {}
    for line in r.splitlines():
        m = re.match(r"^\s*\[\s*(\d+)\]\s+(\S+)\s+\S+\s+([0-9a-f]+)\s+([0-9a-f]+)", line)
        if m:
            secs[int(m.group(1))] = (int(m.group(3), 16), int(m.group(4), 16))
    addr = ndx = None
    for line in r.splitlines():
        f = line.split()
        if len(f) >= 8 and f[7] == kernel + ".kd":
            addr, ndx = int(f[1], 16), int(f[6])
    if addr is None:
        raise KeyError(kernel)
    sec_addr, sec_off = secs[ndx]
    with open(co, "rb") as fh:
        fh.seek(addr - sec_addr + sec_off)
        kd = fh.read(64)
    rsrc3, rsrc1 = struct.unpack_from("<II", kd, 44)
    total = ((rsrc1 & 0x3F) + 1) * 8
    accum = ((rsrc3 & 0x3F) + 1) * 4
    return {"alloc": total, "arch_vgpr": accum, "agpr": total - accum}


def waves_per_simd(vgpr: int, agpr: int) -> int:
    """Waves one SIMD can hold by register budget (gfx950: 512 unified VGPRs per
    lane, arch and acc registers each allocated in granules of 8)."""
    g = lambda x: (x + 7) // 8 * 8  # noqa: E731
    return max(0, min(8, 512 // max(8, g(vgpr) + g(agpr))))
