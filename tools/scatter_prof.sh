# Kernel traces of tools/scatter_ab.py for each library variant in $VARIANTS
# ("main" = the in-tree library) -> gpurun_out/sprof_<variant> (dev tool).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in ${VARIANTS:-main}; do
  rm -rf gpurun_out/sprof_$V
  if [ $V = main ]; then unset PCFM_LIB; else export PCFM_LIB=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_$V.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sprof_$V -o t -- python tools/scatter_ab.py $V > gpurun_out/sprof_$V.json 2> gpurun_out/sprof_$V.err
done
