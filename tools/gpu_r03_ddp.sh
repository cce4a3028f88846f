# DDP gradient-mean test repeated, plain and with switches, to locate the
# occasional unreproducible head_out.weight gradient
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  tag=$1; shift
  env "$@" PCFM_REPORT=gpurun_out/ddp_$tag.json timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp.py -m gpu -q -k grad_is_mean --timeout 280 --timeout-method thread > gpurun_out/ddp_$tag.log 2>&1
  echo "$tag rc=$?"
}
run base1 A=1
run base2 A=1
run base3 A=1
run noocc1 PCFM_CONV_OCC=0
run noocc2 PCFM_CONV_OCC=0
run noplans1 PCFM_SHARE_PLANS=0
run noplans2 PCFM_SHARE_PLANS=0
