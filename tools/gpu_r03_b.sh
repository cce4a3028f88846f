set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_REPORT=gpurun_out/parity_b.json timeout -k 10 900 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_pvconv.py tests/test_gpu_conv3d.py tests/test_gpu_train_golden.py tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_b.log 2>&1 || echo "PYTEST FAILED rc=$?"
PCFM_CONV_OCC=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-chamfer > gpurun_out/bench_occ0.json 2> gpurun_out/bench_occ0.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-chamfer > gpurun_out/bench_occ1.json 2> gpurun_out/bench_occ1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b -o t -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-chamfer --profile-steps 0 --no-event-timing > gpurun_out/bench_prof_b.json 2> gpurun_out/bench_prof_b.err
