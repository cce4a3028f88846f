# Same-box A/B of library variants (make variant NAME=...): bench.py with each
# libpcfm_<name>.so in $VARIANTS and the main build, twice each, alternating.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab_lib.jsonl
for rep in 1 2; do
  for V in main ${VARIANTS}; do
    if [ $V = main ]; then unset PCFM_LIB; else export PCFM_LIB=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_$V.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-chamfer --steps 20 > gpurun_out/ab_one.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print(json.dumps({'lib': '$V', 'ms': d['ms_per_step']}))" >> gpurun_out/ab_lib.jsonl
  done
done
