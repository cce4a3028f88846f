# film backward with recomputed u + devox in-range fast path: tests, A/B, gather PMC, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_devchk.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_pvconv.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fa.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_fa.log; exit 1; }
tail -2 gpurun_out/pytest_fa.log
rm -f /tmp/scat_fa.pt
for rep in 1 2; do
  SCATTER_SAVE=/tmp/scat_fa.pt timeout -k 10 120 python tools/scatter_ab.py main >> gpurun_out/scat_fa.jsonl 2>> gpurun_out/scat_fa.err || exit $?
  SCATTER_SAVE=/tmp/scat_fa.pt PCFM_LIB=$V timeout -k 10 120 python tools/scatter_ab.py devchk >> gpurun_out/scat_fa.jsonl 2>> gpurun_out/scat_fa.err || exit $?
done
echo "ab ok"
mkdir -p gpurun_out/kpmc_fa
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d gpurun_out/kpmc_fa/p$i -o t -- python tools/kernel_pmc.py run > gpurun_out/kpmc_fa/p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python tools/kernel_pmc.py summarize gpurun_out/kpmc_fa/p1 gpurun_out/kpmc_fa/p2 > gpurun_out/kernel_pmc_fa.json
echo "kpmc ok"
timeout -k 10 300 python bench.py > gpurun_out/bench_fa.json 2> gpurun_out/bench_fa.err || { echo "bench failed"; tail -20 gpurun_out/bench_fa.err; exit 1; }
cat gpurun_out/bench_fa.json
