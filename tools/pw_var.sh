set -e
cd $GRAFT_REPO_ROOT
: > gpurun_out/pw_var.jsonl
for V in main ${VARIANTS}; do
  if [ $V = main ]; then unset PCFM_LIB; else export PCFM_LIB=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_$V.so; fi
  timeout -k 10 120 python tools/pw_tail.py $V >> gpurun_out/pw_var.jsonl 2>/dev/null
done
