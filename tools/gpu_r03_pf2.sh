# streaming pointwise GEMM: one vs two chunks of B-operand prefetch, with and
# without the 128-row M slices for M > 128
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
VD=$PWD/point-cloud-flow-matching_amd/csrc/build/variants
rm -f /tmp/pw_pf.pt
for rep in 1 2; do
  PW_SAVE=/tmp/pw_pf.pt timeout -k 10 120 python tools/pw_ab.py main >> gpurun_out/pw_pf.jsonl 2>> gpurun_out/pw_pf.err || exit $?
  PW_SAVE=/tmp/pw_pf.pt PCFM_LIB=$VD/libpcfm_pf2.so timeout -k 10 120 python tools/pw_ab.py pf2 >> gpurun_out/pw_pf.jsonl 2>> gpurun_out/pw_pf.err || exit $?
  PCFM_PW_STREAM_M=1 timeout -k 10 120 python tools/pw_ab.py main_sm >> gpurun_out/pw_pf.jsonl 2>> gpurun_out/pw_pf.err || exit $?
  PCFM_PW_STREAM_M=1 PCFM_LIB=$VD/libpcfm_pf2.so timeout -k 10 120 python tools/pw_ab.py pf2_sm >> gpurun_out/pw_pf.jsonl 2>> gpurun_out/pw_pf.err || exit $?
done
timeout -k 10 300 env PCFM_LIB=$VD/libpcfm_pf2.so python -u -m pytest tests/test_gpu_pointwise.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pf.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_pf.log
cat gpurun_out/pw_pf.jsonl
