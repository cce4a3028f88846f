# Counter passes over tools/kernel_pmc.py (one rocprofv3 run per counter set,
# within the per-block limits: <= 8 SQ, <= 2 GRBM), then the summary ->
# gpurun_out/kernel_pmc.json (copy to profiles/).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/kpmc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/kpmc/counters_avail.txt 2>&1 || true
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d gpurun_out/kpmc/p$i -o t -- python tools/kernel_pmc.py run > gpurun_out/kpmc/p$i.log 2>&1
done
python tools/kernel_pmc.py summarize gpurun_out/kpmc/p1 gpurun_out/kpmc/p2 > gpurun_out/kernel_pmc.json
