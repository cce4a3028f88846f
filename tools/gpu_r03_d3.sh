cd $GRAFT_REPO_ROOT
bash tools/gpu_r03_d2.sh
echo "d2 rc $?"
bash tools/gpu_profile.sh
echo "profile rc $?"
python tools/kgaps.py "$(ls gpurun_out/prof/*/t_kernel_trace.csv 2>/dev/null | head -1 || ls gpurun_out/prof/t_kernel_trace.csv)" 5 > gpurun_out/kgaps.json
