# Two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over tools/op_traffic.py,
# then the per-launch summary -> gpurun_out/traffic.json (copy to profiles/).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rm -rf gpurun_out/pmc/fetch gpurun_out/pmc/write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o t -- python tools/op_traffic.py run > gpurun_out/pmc/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o t -- python tools/op_traffic.py run > gpurun_out/pmc/write.log 2>&1
python tools/op_traffic.py summarize gpurun_out/pmc/fetch gpurun_out/pmc/write > gpurun_out/traffic.json
