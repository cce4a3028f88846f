# devox backward tile forms under rocprofv3 (dev): quad (default) and column (PCFM_DEVOX_QUAD=0)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -rf gpurun_out/sq gpurun_out/sc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sq -o q -- python tools/scatter_ab.py quad > gpurun_out/sq.json
PCFM_DEVOX_QUAD=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sc -o c -- python tools/scatter_ab.py col > gpurun_out/sc.json
