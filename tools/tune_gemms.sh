# Re-measure the library GEMM choices of the train step (PyTorch TunableOp) on an
# MI355X and write them to gpurun_out/tunableop_gfx950.csv; copy that file to
# point-cloud-flow-matching_amd/pcfm/data/ (Trainer loads it with tuning off).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/tunableop_gfx950.csv
PCFM_TUNE_GEMMS=gpurun_out/tunableop_gfx950.csv timeout -k 10 600 python bench.py --steps 2 --warmup 2 \
  --no-cpu-baseline --no-chamfer --no-event-timing > gpurun_out/tune.json 2> gpurun_out/tune.err
