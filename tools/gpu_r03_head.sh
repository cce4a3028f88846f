# HEAD validation: the whole -m gpu suite, smoke and the default bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_REPORT=gpurun_out/parity_head.json timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_head.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_head.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_head.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 python bench.py > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/bench_head.json')); print(d['ms_per_step'], d['value'])"
