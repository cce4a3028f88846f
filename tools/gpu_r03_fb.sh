# film backward: constants in LDS + recomputed u vs the previous form
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_filmold.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fb.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_fb.log; exit 1; }
tail -1 gpurun_out/pytest_fb.log
for rep in 1 2; do
  timeout -k 10 120 python tools/film_ab.py main >> gpurun_out/film_fb.jsonl 2>> gpurun_out/film_fb.err || exit $?
  PCFM_LIB=$V timeout -k 10 120 python tools/film_ab.py filmold >> gpurun_out/film_fb.jsonl 2>> gpurun_out/film_fb.err || exit $?
done
cat gpurun_out/film_fb.jsonl
