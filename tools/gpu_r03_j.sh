cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PCFM_CONV_PP=0 timeout -k 10 300 python tools/conv_pp_check.py gpurun_out/conv_pp0.pt > gpurun_out/conv_pp0.jsonl 2> gpurun_out/conv_pp0.err || exit $?
PCFM_CONV_PP=1 timeout -k 10 300 python tools/conv_pp_check.py gpurun_out/conv_pp1.pt > gpurun_out/conv_pp1.jsonl 2> gpurun_out/conv_pp1.err || exit $?
python tools/conv_pp_check.py --compare gpurun_out/conv_pp0.pt gpurun_out/conv_pp1.pt > gpurun_out/conv_pp_cmp.json
rm -f gpurun_out/conv_pp0.pt gpurun_out/conv_pp1.pt
PCFM_CONV_PP=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-chamfer > gpurun_out/bench_pp1.json 2> gpurun_out/bench_pp1.err
