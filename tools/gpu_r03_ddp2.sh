# DDP gradient-mean test with the per-op checksum trace, repeated
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  PCFM_DDP_TRACE=1 PCFM_REPORT=gpurun_out/ddp_tr$i.json timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp.py -m gpu -q -k grad_is_mean --timeout 280 --timeout-method thread > gpurun_out/ddp_tr$i.log 2>&1
  echo "tr$i rc=$?"
done
