# Default bench (no CPU leg) + a kernel-trace profile of 10 steps and the
# per-step breakdown -> gpurun_out/{bench.json,prof/,breakdown.txt}
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --no-chamfer > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o t -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
python tools/step_breakdown.py "$(ls gpurun_out/prof/*/t_kernel_trace.csv 2>/dev/null | head -1 || ls gpurun_out/prof/t_kernel_trace.csv)" 5 70 > gpurun_out/breakdown.txt
