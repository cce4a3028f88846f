# 16x16x32 weight-gradient form (variant wmf16): timings and the conv tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_wmf16.so
for rep in 1 2; do
  timeout -k 10 120 python tools/conv_ab.py main >> gpurun_out/convab_z.jsonl 2>> gpurun_out/convab_z.err || exit $?
  PCFM_LIB=$V timeout -k 10 120 python tools/conv_ab.py wmf16 >> gpurun_out/convab_z.jsonl 2>> gpurun_out/convab_z.err || exit $?
done
PCFM_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3d.py tests/test_gpu_pvconv.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_z.log 2>&1
echo "pytest rc=$?"
