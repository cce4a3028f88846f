# Voxel-list form of PVConv's first conv: tests, then bench A/B
# (PCFM_CONV_VLIST 0 / 1; list tiles PCFM_CONV_LIST_GN 256 / auto)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_REPORT=gpurun_out/parity_vl.json timeout -k 10 400 python -u -m pytest tests/test_gpu_pvconv.py tests/test_gpu_conv3d.py tests/test_gpu_model.py tests/test_gpu_train_golden.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_vl.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for s in 0 1 2; do
    case $s in 0) E="PCFM_CONV_VLIST=0";; 1) E="PCFM_CONV_LIST_GN=256";; 2) E="PCFM_CONV_LIST_GN=auto";; esac
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-chamfer --steps 20 --warmup 5 > gpurun_out/bench_vl_s$s.$rep.json 2>/dev/null || exit $?
  done
done
echo bench done
