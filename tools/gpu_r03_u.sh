# A/B of the 16x16x32-MFMA form of the voxel-conv GEMM (variant mf16) against
# the main build: kernel timings, the conv tests on the variant, bench A/B.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_mf16.so
timeout -k 10 120 python tools/conv_ab.py main > gpurun_out/convab_u.jsonl 2> gpurun_out/convab_u.err || exit $?
PCFM_LIB=$V timeout -k 10 120 python tools/conv_ab.py mf16 >> gpurun_out/convab_u.jsonl 2>> gpurun_out/convab_u.err || exit $?
timeout -k 10 120 python tools/conv_ab.py main >> gpurun_out/convab_u.jsonl 2>> gpurun_out/convab_u.err || exit $?
PCFM_LIB=$V timeout -k 10 120 python tools/conv_ab.py mf16 >> gpurun_out/convab_u.jsonl 2>> gpurun_out/convab_u.err || exit $?
echo convab done
PCFM_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3d.py tests/test_gpu_pvconv.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_u.log 2>&1
echo "pytest rc=$?"
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-chamfer --steps 20 --warmup 5 > gpurun_out/bench_u_main$rep.json 2>/dev/null || exit $?
  PCFM_LIB=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-chamfer --steps 20 --warmup 5 > gpurun_out/bench_u_mf16$rep.json 2>/dev/null || exit $?
done
echo bench done
