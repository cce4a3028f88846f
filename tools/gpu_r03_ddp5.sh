# DDP gradient-mean test with device-coherent loads of the devoxelization's
# `add` operand (variant coh), repeated
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out

for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  PCFM_DDP_TRACE=1 PCFM_REPORT=gpurun_out/ddp_stag$i.json timeout -k 10 200 python -u -m pytest tests/test_gpu_ddp.py -m gpu -q -k grad_is_mean --timeout 190 --timeout-method thread > gpurun_out/ddp_stag$i.log 2>&1
  echo "stag$i rc=$?"
done
