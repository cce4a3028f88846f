# head weight gradient: occupancy / split-count A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
VD=$PWD/point-cloud-flow-matching_amd/csrc/build/variants
for rep in 1 2; do
  timeout -k 10 120 python tools/rows_ab.py main >> gpurun_out/rows_ab.jsonl 2>> gpurun_out/rows_ab.err || exit $?
  PCFM_LIB=$VD/libpcfm_rw3.so PCFM_RW_BPC=3 timeout -k 10 120 python tools/rows_ab.py rw3 >> gpurun_out/rows_ab.jsonl 2>> gpurun_out/rows_ab.err || exit $?
  PCFM_LIB=$VD/libpcfm_rw3.so PCFM_RW_BPC=6 timeout -k 10 120 python tools/rows_ab.py rw3 >> gpurun_out/rows_ab.jsonl 2>> gpurun_out/rows_ab.err || exit $?
  PCFM_LIB=$VD/libpcfm_rw4.so PCFM_RW_BPC=4 timeout -k 10 120 python tools/rows_ab.py rw4 >> gpurun_out/rows_ab.jsonl 2>> gpurun_out/rows_ab.err || exit $?
  PCFM_RW_BPC=4 timeout -k 10 120 python tools/rows_ab.py main >> gpurun_out/rows_ab.jsonl 2>> gpurun_out/rows_ab.err || exit $?
done
cat gpurun_out/rows_ab.jsonl
