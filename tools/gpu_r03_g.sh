cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_REPORT=gpurun_out/parity_g.json timeout -k 10 600 python -u -m pytest tests/test_gpu_conv3d.py tests/test_gpu_norm.py tests/test_gpu_pvconv.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_g.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-chamfer > gpurun_out/bench_g.json 2> gpurun_out/bench_g.err || exit $?
REPS=30 timeout -k 10 400 python tools/op_det_probe.py > gpurun_out/opdet0.jsonl 2> gpurun_out/opdet0.err &
p0=$!
REPS=30 timeout -k 10 400 python tools/op_det_probe.py > gpurun_out/opdet1.jsonl 2> gpurun_out/opdet1.err &
p1=$!
wait $p0; r0=$?
wait $p1; r1=$?
echo "probe rc $r0 $r1"
