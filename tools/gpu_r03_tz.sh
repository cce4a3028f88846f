cd $GRAFT_REPO_ROOT
bash tools/gpu_r03_t.sh
echo "t done"
bash tools/gpu_r03_z.sh
echo "z done"
