# Same-box bench A/B of library variants (dev tool): $VARIANTS built by
# `make variant`, "main" = the in-tree library; bench.py twice each, alternating.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/lib_ab.jsonl
for rep in 1 2; do
  for V in main ${VARIANTS}; do
    if [ $V = main ]; then unset PCFM_LIB; else export PCFM_LIB=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_$V.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/lib_one.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/lib_one.json')); print(json.dumps({'lib': '$V', 'ms': d['ms_per_step']}))" >> gpurun_out/lib_ab.jsonl
  done
done
