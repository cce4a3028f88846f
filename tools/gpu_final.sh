# Round-end refresh: gpu tests, smoke, default bench, kernel-trace profile,
# C5 train bench and the bf16 Heun sampling bench (copy results to profiles/).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_round.sh
timeout -k 10 300 python bench.py --batch 4 --points 100000 --steps 5 --warmup 2 --no-cpu-baseline --no-chamfer > gpurun_out/c5_train.json 2> gpurun_out/c5_train.err
timeout -k 10 300 python tools/sample_bench.py --amp > gpurun_out/sample_amp.json 2> gpurun_out/sample_amp.err
