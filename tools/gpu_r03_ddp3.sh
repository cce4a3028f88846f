# DDP gradient-mean test repeated with the no-streamed-access build (PCFM_NT=0)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_nont.so
for i in 1 2 3 4 5 6; do
  PCFM_DDP_TRACE=1 PCFM_REPORT=gpurun_out/ddp_nt$i.json timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp.py -m gpu -q -k grad_is_mean --timeout 280 --timeout-method thread > gpurun_out/ddp_nt$i.log 2>&1
  echo "nt$i rc=$?"
done
