cd $GRAFT_REPO_ROOT
bash tools/gpu_r03_i.sh
