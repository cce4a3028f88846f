# pointwise weight gradient: blocks per CU A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
VD=$PWD/point-cloud-flow-matching_amd/csrc/build/variants
rm -f /tmp/pw_wg.pt
for rep in 1 2; do
  PW_SAVE=/tmp/pw_wg.pt timeout -k 10 120 python tools/pw_ab.py main >> gpurun_out/pw_wg.jsonl 2>> gpurun_out/pw_wg.err || exit $?
  PW_SAVE=/tmp/pw_wg.pt PCFM_LIB=$VD/libpcfm_wg3.so timeout -k 10 120 python tools/pw_ab.py wg3 >> gpurun_out/pw_wg.jsonl 2>> gpurun_out/pw_wg.err || exit $?
  PW_SAVE=/tmp/pw_wg.pt PCFM_LIB=$VD/libpcfm_wg4.so timeout -k 10 120 python tools/pw_ab.py wg4 >> gpurun_out/pw_wg.jsonl 2>> gpurun_out/pw_wg.err || exit $?
done
cat gpurun_out/pw_wg.jsonl
