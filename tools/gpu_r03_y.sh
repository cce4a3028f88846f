cd $GRAFT_REPO_ROOT
bash tools/gpu_r03_u.sh || exit $?
echo "u done"
bash tools/gpu_r03_v.sh || exit $?
echo "v done"
bash tools/gpu_r03_x.sh || exit $?
echo "x done"
