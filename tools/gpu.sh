# The one GPU-box runner: bash tools/gpu.sh TASK [TASK ...]   (via gpurun)
#
# Every task runs under its own time limit; the first failure ends the call
# (set -e), so nothing else touches the GPU after a fault, abort or timeout.
#
#   tests     full -m gpu suite, parity report  -> gpurun_out/pytest_gpu.log, parity.json
#   quick     $TESTS (default tests/test_gpu_ops.py) -x -q  -> gpurun_out/pytest_quick.log,
#             parity_quick.json
#   smoke     __graft_entry__.smoke()           -> gpurun_out/smoke.log
#   bench     default bench.py (+ $BENCH_ARGS)  -> gpurun_out/bench.json / .err
#   benchq    bench.py without the CPU / Chamfer legs  -> gpurun_out/benchq.json
#   prof      rocprofv3 --kernel-trace --stats of 10 bench steps + per-step
#             breakdown -> gpurun_out/prof/, gpurun_out/breakdown.txt
#   kpmc      MFMA / LDS / wait counters of the conv kernels (tools/kernel_pmc.sh)
#   traffic   FETCH_SIZE / WRITE_SIZE passes of the voxel ops (tools/pmc_traffic.sh)
#   c5        bench.py at B=4, N=100000     -> gpurun_out/c5_train.json
#   sample    bf16 Heun / dopri5 sampling bench  -> gpurun_out/sample_amp.json
#   ddp       the two-rank DDP tests, ranks concurrent on the one GPU, with the
#             devoxelization self-check on   -> gpurun_out/ddp_check.log
#   ab        bench.py (quick form) once per variant of $AB, a space-separated list
#             of NAME or NAME:VAR=V,VAR2=V2 (env for that run; NAME alone = defaults)
#             -> gpurun_out/ab.jsonl (ms/step, roofline frac, per-op ms)
#   script:F  run python F (a measurement script of tools/) -> gpurun_out/F.jsonl
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCHQ="--no-cpu-baseline --no-chamfer"
for task in "$@"; do
  echo "[gpu.sh] $task $(date +%T)"
  case "$task" in
    tests)
      PCFM_REPORT=gpurun_out/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v \
        --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ;;
    quick)
      PCFM_REPORT=gpurun_out/parity_quick.json timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_ops.py} -m gpu -x -v \
        --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench)
      timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err ;;
    benchq)
      timeout -k 10 300 python bench.py $BENCHQ ${BENCH_ARGS:-} > gpurun_out/benchq.json 2> gpurun_out/benchq.err ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o t \
        -- python bench.py --steps 10 --warmup 3 $BENCHQ > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
      python tools/step_breakdown.py "$(ls gpurun_out/prof/*/t_kernel_trace.csv gpurun_out/prof/t_kernel_trace.csv 2>/dev/null | head -1)" 5 90 \
        > gpurun_out/breakdown.txt ;;
    kpmc)
      bash tools/kernel_pmc.sh ;;
    traffic)
      bash tools/pmc_traffic.sh ;;
    c5)
      timeout -k 10 300 python bench.py --batch 4 --points 100000 --steps 5 --warmup 2 $BENCHQ \
        > gpurun_out/c5_train.json 2> gpurun_out/c5_train.err ;;
    sample)
      timeout -k 10 300 python tools/sample_bench.py --amp > gpurun_out/sample_amp.json 2> gpurun_out/sample_amp.err ;;
    ddp)
      PCFM_DEVOX_VERIFY=1 timeout -k 10 400 python -u -m pytest \
        tests/test_gpu_ddp.py -m gpu -v -rxX --timeout 300 --timeout-method thread \
        > gpurun_out/ddp_check.log 2>&1 ;;
    ab)
      : > gpurun_out/ab.jsonl
      for v in ${AB:-base}; do
        name="${v%%:*}"; envs=""
        [ "$name" != "$v" ] && envs="${v#*:}" && envs="${envs//,/ }"
        env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 3 $BENCHQ \
          > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err
        python -c "import json,sys; d=json.load(open('gpurun_out/ab_one.json')); print(json.dumps({'v': sys.argv[1], 'ms': d['ms_per_step'], 'frac': d['roofline']['frac'], 'ops': {k: round(v['ms_per_step'], 4) for k, v in d['kernels'].items()}}))" "$v" >> gpurun_out/ab.jsonl
      done ;;
    script:*)
      f="${task#script:}"
      timeout -k 10 400 python "$f" ${SCRIPT_ARGS:-} > "gpurun_out/$(basename "$f" .py).jsonl" \
        2> "gpurun_out/$(basename "$f" .py).err" ;;
    *)
      echo "unknown task $task" >&2; exit 2 ;;
  esac
done
echo "[gpu.sh] done $(date +%T)"
