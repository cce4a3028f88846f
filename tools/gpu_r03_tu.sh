cd $GRAFT_REPO_ROOT
bash tools/gpu_r03_u.sh || exit $?
echo "u done"
bash tools/gpu_r03_t.sh
