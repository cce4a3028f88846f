# Round-3 measurement set, part C: PMC traffic + MFMA counters, then the
# default bench line and its rocprofv3 kernel-trace --stats run
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_traffic.sh || exit $?
echo traffic ok
bash tools/kernel_pmc.sh || exit $?
echo kpmc ok
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
echo bench ok
rm -rf gpurun_out/prof_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o t -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/bench_prof_final.json 2> gpurun_out/bench_prof_final.err || exit $?
echo prof ok
