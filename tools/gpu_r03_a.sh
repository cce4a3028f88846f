set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_REPORT=gpurun_out/parity_a.json timeout -k 10 900 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_optim.py "tests/test_gpu_ops.py::test_chamfer_c2_product_path" tests/test_gpu_train_golden.py tests/test_gpu_model.py tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_a.log 2>&1 || echo "PYTEST FAILED rc=$?"
PCFM_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-chamfer --no-event-timing > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err
