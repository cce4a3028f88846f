set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pointwise.py tests/test_gpu_model.py tests/test_gpu_head.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 120 python tools/pw_ab.py main > gpurun_out/pw_main.json
PCFM_LIB=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_nostream.so timeout -k 10 120 python tools/pw_ab.py nostream > gpurun_out/pw_nostream.json
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/bench_main.json 2>/dev/null
PCFM_LIB=$PWD/point-cloud-flow-matching_amd/csrc/build/variants/libpcfm_nostream.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/bench_nostream.json 2>/dev/null
