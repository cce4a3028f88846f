# Forward reproducibility: solo module-level probe, then the op-level trace
# under contention (two processes on the one GPU, as the DDP rehearsal runs)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/poison_probe.py > gpurun_out/poison_t.jsonl 2> gpurun_out/poison_t.err
echo "poison rc $?"
RUNS=6 timeout -k 10 300 python tools/det_forward_probe.py > gpurun_out/detfwd_t.jsonl 2> gpurun_out/detfwd_t.err || exit $?
echo solo done
RUNS=8 timeout -k 10 400 python tools/det_ops_trace.py > gpurun_out/optrace_t0.jsonl 2> gpurun_out/optrace_t0.err &
p0=$!
RUNS=8 timeout -k 10 400 python tools/det_ops_trace.py > gpurun_out/optrace_t1.jsonl 2> gpurun_out/optrace_t1.err &
p1=$!
wait $p0; r0=$?
wait $p1; r1=$?
echo "probe rc $r0 $r1"
