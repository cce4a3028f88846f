# Round-4 A/B of the conv slab form, BN statistics from the GEMM and the EMD
# phase form: their tests, then bench.py per switch (-> gpurun_out/slab_ab.jsonl)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_REPORT=gpurun_out/ab_report.json timeout -k 10 500 python -u -m pytest tests/test_gpu_conv3d.py tests/test_gpu_norm.py -m gpu -x -v -k "slab or bn_stats_from_gemm or fwd_bwd_vs_fp64 or pair or fused" --timeout 180 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
PCFM_REPORT=gpurun_out/emd_report.json timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v -k "emd" --timeout 120 --timeout-method thread > gpurun_out/pytest_emd.log 2>&1
: > gpurun_out/slab_ab.jsonl
for S in 0 1; do
  PCFM_CONV_SLAB=$S timeout -k 10 120 python tools/conv_ab.py slab$S >> gpurun_out/slab_ab.jsonl
done
for V in new slab0 bnsep new; do
  case $V in
    new) E="" ;; slab0) E="PCFM_CONV_SLAB=0" ;; bnsep) E="PCFM_BN_FROM_GEMM=0" ;;
  esac
  env $E timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/lib_one.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/lib_one.json')); print(json.dumps({'v': '$V', 'ms': d['ms_per_step'], 'frac': d['roofline']['frac'], 'kern': {k: v['ms_per_step'] for k, v in d['kernels'].items() if k.startswith(('conv3d', 'bn', 'pointwise'))}}))" >> gpurun_out/slab_ab.jsonl
done
