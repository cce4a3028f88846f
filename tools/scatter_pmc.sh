# PMC counter passes over tools/scatter_ab.py for each library variant in
# $VARIANTS ("main" = the in-tree library) -> gpurun_out/spmc_<variant>_p<i> (dev tool).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for V in ${VARIANTS:-main}; do
  if [ $V = main ]; then unset PCFM_LIB; else export PCFM_LIB=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_$V.so; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    rm -rf gpurun_out/spmc_${V}_p$i
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/spmc_${V}_p$i -o t -- python tools/scatter_ab.py $V > gpurun_out/spmc_${V}_p$i.log 2>&1
  done
done
