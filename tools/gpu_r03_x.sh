# M-sliced streaming pointwise GEMM (PCFM_PW_STREAM_M=1) vs the 256-row tile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/pw_ref.pt
for s in 0 1 0 1; do
  PCFM_PW_STREAM_M=$s PW_SAVE=gpurun_out/pw_ref.pt timeout -k 10 120 python tools/pw_ab.py s$s >> gpurun_out/pwab_x.jsonl 2>> gpurun_out/pwab_x.err || exit $?
done
rm -f gpurun_out/pw_ref.pt
echo pw done
for rep in 1 2; do
  for s in 0 1; do
    PCFM_PW_STREAM_M=$s timeout -k 10 200 python bench.py --no-cpu-baseline --no-chamfer --steps 20 --warmup 5 > gpurun_out/bench_x_s$s.$rep.json 2>/dev/null || exit $?
  done
done
echo bench done
