# Kernel traces of the bench step under two environments ($A, $B: "NAME=VALUE"
# or "base") -> gpurun_out/prof_A, gpurun_out/prof_B (dev tool).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_A gpurun_out/prof_B
i=0
for E in "$A" "$B"; do
  i=$((i+1)); tag=$([ $i = 1 ] && echo A || echo B)
  if [ "$E" = base ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$tag -o t -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/prof_$tag.json 2>/dev/null
  else
    export $E
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$tag -o t -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-chamfer > gpurun_out/prof_$tag.json 2>/dev/null
    unset ${E%%=*}
  fi
done
