# Round-3 measurement set, part A: the whole -m gpu suite with its parity
# report, smoke, the default bench line (CPU baseline, Chamfer / EMD legs) and
# a rocprofv3 kernel-trace --stats run of the same bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_REPORT=gpurun_out/parity_final.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
echo bench ok
rm -rf gpurun_out/prof_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o t -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/bench_prof_final.json 2> gpurun_out/bench_prof_final.err || exit $?
echo prof ok
