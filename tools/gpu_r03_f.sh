# two concurrent processes on the one GPU (as the DDP rehearsal runs): does
# contention expose a race in the point flow's forward?
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
RUNS=8 timeout -k 10 400 python tools/det_forward_probe.py > gpurun_out/det_con0.jsonl 2> gpurun_out/det_con0.err &
p0=$!
RUNS=8 timeout -k 10 400 python tools/det_forward_probe.py > gpurun_out/det_con1.jsonl 2> gpurun_out/det_con1.err &
p1=$!
wait $p0; r0=$?
wait $p1; r1=$?
echo "rc $r0 $r1"
[ $r0 -eq 0 ] && [ $r1 -eq 0 ]
