cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
RUNS=8 timeout -k 10 400 python tools/det_ops_trace.py > gpurun_out/optrace0.jsonl 2> gpurun_out/optrace0.err &
p0=$!
RUNS=8 timeout -k 10 400 python tools/det_ops_trace.py > gpurun_out/optrace1.jsonl 2> gpurun_out/optrace1.err &
p1=$!
wait $p0; r0=$?
wait $p1; r1=$?
echo "probe rc $r0 $r1"
