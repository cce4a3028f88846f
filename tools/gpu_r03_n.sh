cd $GRAFT_REPO_ROOT
bash tools/gpu_r03_m.sh
echo "m done"
bash tools/gpu_r03_i.sh
