set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in main ${VARIANTS}; do
  if [ $V = main ]; then unset PCFM_LIB; else export PCFM_LIB=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_$V.so; fi
  rm -rf gpurun_out/sp_$V
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sp_$V -o t -- python tools/scatter_ab.py $V > gpurun_out/sp_$V.log 2>&1
done
