set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3d.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
: > gpurun_out/slab_ab.jsonl
for rep in 1 2; do
  for S in 0 1; do
    PCFM_CONV_SLAB=$S timeout -k 10 120 python tools/conv_ab.py slab$S >> gpurun_out/slab_ab.jsonl
    PCFM_CONV_SLAB=$S timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/lib_one.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/lib_one.json')); print(json.dumps({'slab': $S, 'ms': d['ms_per_step'], 'frac': d['roofline']['frac']}))" >> gpurun_out/slab_ab.jsonl
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v -k "emd" --timeout 120 --timeout-method thread > gpurun_out/pytest_emd.log 2>&1
PCFM_REPORT=gpurun_out/emd_report.json timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k "emd_phase" --timeout 120 --timeout-method thread >> gpurun_out/pytest_emd.log 2>&1
