# Full GPU test suite with the parity report (gpurun_out/parity.json), then a
# short bench line.  Usage (on the box): bash tools/gpu_tests.sh [pytest args]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_REPORT=gpurun_out/parity.json timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
