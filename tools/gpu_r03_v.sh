# Unit-gather channel groups per wave (PCFM_SEG_GROUPS 1 / 2 / 4): scatter
# timings at the C2 stage shapes, bitwise equality across the settings, the
# scatter tests, bench A/B.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/scat_ref.pt
for g in 1 2 4 1 2 4; do
  PCFM_SEG_GROUPS=$g SCATTER_SAVE=gpurun_out/scat_ref.pt timeout -k 10 120 python tools/scatter_ab.py g$g >> gpurun_out/scatab_v.jsonl 2>> gpurun_out/scatab_v.err || exit $?
done
rm -f gpurun_out/scat_ref.pt
echo scatter done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_pvconv.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_v.log 2>&1
echo "pytest rc=$?"
for rep in 1 2; do
  for g in 1 2 4; do
    PCFM_SEG_GROUPS=$g timeout -k 10 200 python bench.py --no-cpu-baseline --no-chamfer --steps 20 --warmup 5 > gpurun_out/bench_v_g$g.$rep.json 2>/dev/null || exit $?
  done
done
echo bench done
