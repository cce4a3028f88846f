cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_CONV_BRICK=0 timeout -k 10 300 python tools/conv_pp_check.py gpurun_out/conv_b0.pt > gpurun_out/conv_b0.jsonl 2> gpurun_out/conv_b0.err || exit $?
PCFM_CONV_BRICK=1 timeout -k 10 300 python tools/conv_pp_check.py gpurun_out/conv_b1.pt > gpurun_out/conv_b1.jsonl 2> gpurun_out/conv_b1.err || exit $?
python tools/conv_pp_check.py --compare gpurun_out/conv_b0.pt gpurun_out/conv_b1.pt > gpurun_out/conv_b_cmp.json
rm -f gpurun_out/conv_b0.pt gpurun_out/conv_b1.pt
PCFM_REPORT=gpurun_out/parity_m.json timeout -k 10 600 python -u -m pytest tests/test_gpu_conv3d.py tests/test_gpu_norm.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_m.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-chamfer > gpurun_out/bench_m.json 2> gpurun_out/bench_m.err
