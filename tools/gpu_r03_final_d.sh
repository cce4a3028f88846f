# Round-3 measurement set at the final tree: the whole -m gpu suite with its
# parity report, smoke, the default bench line, a rocprofv3 kernel-trace --stats
# run of the same bench and the host-enqueue vs device time per step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_REPORT=gpurun_out/parity_r3b.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r3b.log 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3b.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 python bench.py > gpurun_out/bench_r3b.json 2> gpurun_out/bench_r3b.err || exit $?
echo bench ok
rm -rf gpurun_out/prof_r3b
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3b -o t -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/bench_prof_r3b.json 2> gpurun_out/bench_prof_r3b.err || exit $?
echo prof ok
timeout -k 10 180 python tools/host_time.py > gpurun_out/host_time_r3b.txt 2>&1 || exit $?
cat gpurun_out/host_time_r3b.txt
