# The devoxelization gather under contention: two stress processes at once,
# then the op-level trace pair again (with output details)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ITERS=150 timeout -k 10 300 python tools/devox_stress.py > gpurun_out/dstress0.jsonl 2> gpurun_out/dstress0.err &
p0=$!
ITERS=150 SEED=1 timeout -k 10 300 python tools/devox_stress.py > gpurun_out/dstress1.jsonl 2> gpurun_out/dstress1.err &
p1=$!
wait $p0; r0=$?
wait $p1; r1=$?
echo "stress rc $r0 $r1"
[ $r0 -eq 0 ] && [ $r1 -eq 0 ] || exit 1
ITERS=150 timeout -k 10 300 python tools/devox_stress.py > gpurun_out/dstress_solo.jsonl 2> gpurun_out/dstress_solo.err || exit $?
echo "solo done"
RUNS=8 timeout -k 10 400 python tools/det_ops_trace.py > gpurun_out/optrace_d0.jsonl 2> gpurun_out/optrace_d0.err &
p0=$!
RUNS=8 timeout -k 10 400 python tools/det_ops_trace.py > gpurun_out/optrace_d1.jsonl 2> gpurun_out/optrace_d1.err &
p1=$!
wait $p0; r0=$?
wait $p1; r1=$?
echo "trace rc $r0 $r1"
