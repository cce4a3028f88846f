set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_pvconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1
for V in main u1 u4; do
  if [ $V = main ]; then unset PCFM_LIB; else export PCFM_LIB=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_$V.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab/$V -o t -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/ab/$V.json 2> gpurun_out/ab/$V.err
done
