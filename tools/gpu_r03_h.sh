cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/blas_det_probe.py > gpurun_out/blasdet_solo.jsonl 2> gpurun_out/blasdet_solo.err || exit $?
timeout -k 10 400 python tools/blas_det_probe.py > gpurun_out/blasdet0.jsonl 2> gpurun_out/blasdet0.err &
p0=$!
timeout -k 10 400 python tools/blas_det_probe.py > gpurun_out/blasdet1.jsonl 2> gpurun_out/blasdet1.err &
p1=$!
wait $p0; r0=$?
wait $p1; r1=$?
echo "probe rc $r0 $r1"
