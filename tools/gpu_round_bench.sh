# Round-end measurement set: the default bench line (CPU baseline included) and
# a rocprofv3 kernel-trace --stats run of the same command (short) ->
# gpurun_out/{bench_full.json, prof_full/} (copy the summaries to profiles/).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_full -o t -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/bench_prof_full.json 2> gpurun_out/bench_prof_full.err
