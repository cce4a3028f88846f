# bn_ab.py once per library variant ($VARIANTS built by `make variant`; "main" =
# the in-tree library) -> gpurun_out/bn_var.jsonl (dev tool)
set -e
cd $GRAFT_REPO_ROOT
: > gpurun_out/bn_var.jsonl
for V in main ${VARIANTS}; do
  if [ $V = main ]; then unset PCFM_LIB; else export PCFM_LIB=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_$V.so; fi
  timeout -k 10 120 python tools/bn_ab.py $V >> gpurun_out/bn_var.jsonl 2>/dev/null
done
