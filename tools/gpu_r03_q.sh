cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/oob_probe.py > gpurun_out/oob.jsonl 2> gpurun_out/oob.err
echo "oob rc $?"
FREEZE=0 RUNS=10 timeout -k 10 300 python tools/det_forward_probe.py > gpurun_out/det_fwd_nofreeze.jsonl 2> gpurun_out/det_fwd_nofreeze.err
echo "det rc $?"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ddp.py -m gpu > gpurun_out/pytest_ddp.log 2>&1
echo "ddp rc $?"
