# Round-3 measurement set, part B: PMC traffic (FETCH_SIZE / WRITE_SIZE, two
# passes) and the MFMA / LDS counter passes of the conv kernels
cd $GRAFT_REPO_ROOT
bash tools/pmc_traffic.sh || exit $?
echo traffic ok
bash tools/kernel_pmc.sh || exit $?
echo kpmc ok
