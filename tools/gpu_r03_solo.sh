# The DDP test's reference step repeated in ONE process (no GPU contention)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
RUNS=60 timeout -k 10 400 python tools/solo_repeat.py > gpurun_out/solo.jsonl 2> gpurun_out/solo.err
echo "solo rc $?"
