set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/det_forward_probe.py > gpurun_out/det_fwd.jsonl 2> gpurun_out/det_fwd.err
BWD=1 timeout -k 10 300 python tools/det_forward_probe.py > gpurun_out/det_bwd.jsonl 2> gpurun_out/det_bwd.err
