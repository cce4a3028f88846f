cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py -m gpu -k "emd or grid_sample" > gpurun_out/pytest_p.log 2>&1
echo "pytest rc $?"
FREEZE=0 RUNS=10 timeout -k 10 300 python tools/pv_race_probe.py > gpurun_out/pvrace0.jsonl 2> gpurun_out/pvrace0.err &
p0=$!
FREEZE=0 RUNS=10 timeout -k 10 300 python tools/pv_race_probe.py > gpurun_out/pvrace1.jsonl 2> gpurun_out/pvrace1.err &
p1=$!
wait $p0; r0=$?
wait $p1; r1=$?
echo "probe rc $r0 $r1"
