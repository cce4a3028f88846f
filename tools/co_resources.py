"""Per-kernel resources read from code objects (CPU only): LDS, registers the
hardware allocates per lane (kernel descriptor), waves per SIMD by registers and
workgroups per CU by LDS -- for the co-residence analysis of DESIGN.md section 6.

    python tools/co_resources.py [--json]

Reads the in-tree libpcfm_hip.so, torch's librccl.so and the hipBLASLt kernel
the co-residence probe's "blas" aggressor ran (named by rocprofv3 on MI355X:
profiles/r05_blas_kernel.txt)."""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "helpers"))
import codeobj as C  # noqa: E402

LDS_CU = 160 * 1024


def rows(path, patterns, dyn_lds=None):
    dyn_lds = dyn_lds or {}
    out = []
    with tempfile.TemporaryDirectory() as d:
        for co in C.extract(path, d):
            res = C.kernel_resources(co)
            for name, r in res.items():
                for label, pat in patterns.items():
                    if pat(name):
                        reg = C.descriptor_registers(co, name)
                        lds = r.get("lds", 0) + dyn_lds.get(label, 0)
                        waves_wg = max(1, r.get("wg", 64) // 64)
                        wps = min(8, 512 // reg["alloc"])
                        wg_cu = min(LDS_CU // lds if lds else 99, 4 * wps // max(1, waves_wg // 4)
                                    if waves_wg >= 4 else 99)
                        out.append({"kernel": label, "lds_bytes": lds, "threads": r.get("wg"),
                                    "regs_alloc": reg["alloc"], "agpr": reg["agpr"],
                                    "waves_per_simd_by_regs": wps,
                                    "regs_left_on_simd_at_full_occupancy":
                                        512 - wps * reg["alloc"],
                                    "workgroups_per_cu_by_lds": LDS_CU // lds if lds else None})
    return out


def main():
    import torch
    tl = os.path.join(os.path.dirname(torch.__file__), "lib")
    lib = os.path.join(REPO, "point-cloud-flow-matching_amd", "csrc", "libpcfm_hip.so")
    table = rows(lib, {
        "pw_gemm256 (aggressor: corrupts)": lambda n: "pw_gemm256_kernel" in n,
        "conv3_wgrad3 (aggressor: corrupts)": lambda n: "conv3_wgrad3_kernel" in n,
        "conv3_igemm_glds<32,256,3> (clean)": lambda n: "conv3_igemm_glds_kernelILi32ELi256" in n,
        "gather_rows4<ProvDevox> (victim, R16/R8)": lambda n: "gather_rows4_kernelINS_9ProvDevox" in n,
        "gather_rows1<ProvDevox,2> (victim, R32)": lambda n: "gather_rows1_kernelINS_9ProvDevoxELi2" in n,
    }, dyn_lds={"conv3_wgrad3 (aggressor: corrupts)": 2 * (2 * 64 * 256 + 2 * 68 * 256),
                "gather_rows4<ProvDevox> (victim, R16/R8)": 4 * 4096 * 4,
                "gather_rows1<ProvDevox,2> (victim, R32)": 32768 * 4})
    blas_name_file = os.path.join(REPO, "profiles", "r05_blas_kernel.txt")
    if os.path.exists(blas_name_file):
        name = open(blas_name_file).read().strip()
        co = os.path.join(tl, "hipblaslt", "library",
                          "TensileLibrary_BB_BB_HA_Bias_SAV_UA_Type_BB_HPA_Contraction_l_Ailk_"
                          "Bljk_Cijk_Dijk_gfx950.co")
        table += rows(co, {"hipBLASLt bf16 4096^2 MT256x256x64 (clean)": lambda n: n == name})
    table += rows(os.path.join(tl, "librccl.so"), {
        "rcclGenericKernel<1> (RCCL)": lambda n: n.startswith("_Z17rcclGenericKernelILi1ELb0E"),
        "rcclGenericKernel<4> (RCCL)": lambda n: n.startswith("_Z17rcclGenericKernelILi4ELb0E")})
    if "--json" in sys.argv:
        print(json.dumps(table, indent=1))
        return
    for r in table:
        print(f"{r['kernel']:45s} LDS {r['lds_bytes']:7d} B  threads {r['threads']:5d}  "
              f"regs {r['regs_alloc']:3d} (acc {r['agpr']:3d})  waves/SIMD {r['waves_per_simd_by_regs']}  "
              f"regs left {r['regs_left_on_simd_at_full_occupancy']:3d}  "
              f"WG/CU by LDS {r['workgroups_per_cu_by_lds']}")


if __name__ == "__main__":
    main()
