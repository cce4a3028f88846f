# DDP gradient-mean test under AMD_SERIALIZE_KERNEL=3 (every kernel waited for
# before and after): does the devoxelization glitch survive serialisation?
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4 5 6 7 8; do
  AMD_SERIALIZE_KERNEL=3 PCFM_DDP_TRACE=1 PCFM_REPORT=gpurun_out/ddp_ser$i.json timeout -k 10 200 python -u -m pytest tests/test_gpu_ddp.py -m gpu -q -k grad_is_mean --timeout 190 --timeout-method thread > gpurun_out/ddp_ser$i.log 2>&1
  echo "ser$i rc=$?"
done
