# State check at re-entry: the whole -m gpu suite (no -x, so every failure
# shows), smoke, a short bench line, the BN-running-stat OOB probe.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_REPORT=gpurun_out/parity_s.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_s.log 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-chamfer > gpurun_out/bench_s.json 2> gpurun_out/bench_s.err || exit $?
echo bench ok
timeout -k 10 200 python tools/oob_probe.py > gpurun_out/oob_s.jsonl 2> gpurun_out/oob_s.err
echo "oob rc $?"
