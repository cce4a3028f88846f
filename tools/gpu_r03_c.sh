set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/pw_det_probe.py > gpurun_out/pw_det.jsonl 2> gpurun_out/pw_det.err
timeout -k 10 300 python tools/conv_occ_probe.py > gpurun_out/conv_occ.jsonl 2> gpurun_out/conv_occ.err
PCFM_REPORT=gpurun_out/parity_c.json timeout -k 10 600 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_pvconv.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_c.log 2>&1 || echo "PYTEST FAILED rc=$?"
