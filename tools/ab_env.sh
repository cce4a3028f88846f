# Same-box A/B of Python-level switches: bench.py under each "NAME=VALUE" in
# $ENVS (space separated; "base" = no change), twice each, alternating.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab_env.jsonl
for rep in ${REPS:-1 2}; do
  for E in base ${ENVS}; do
    if [ $E = base ]; then
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-chamfer --steps 20 > gpurun_out/ab_one.json 2>/dev/null
    else
      timeout -k 10 200 env $E python bench.py --no-cpu-baseline --no-chamfer --steps 20 > gpurun_out/ab_one.json 2>/dev/null
    fi
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_one.json')); print(json.dumps({'env': '$E', 'ms': d['ms_per_step']}))" >> gpurun_out/ab_env.jsonl
  done
done
