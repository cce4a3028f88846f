# voxel-conv weight-gradient decomposition A/B (dev): bash tools/wg_dec.sh <variant names...>
# (PCFM_WGRAD3P selects the form the variants are built for; default the one-wave form)
set -e
V=point-cloud-flow-matching_amd/csrc/build/variants
OUT=gpurun_out/wg_dec.jsonl
timeout -k 10 120 python tools/conv_ab.py main > $OUT
PCFM_WGRAD3P=0 timeout -k 10 120 python tools/conv_ab.py main_12wave >> $OUT
for n in "$@"; do
  PCFM_LIB=$V/libpcfm_$n.so timeout -k 10 120 python tools/conv_ab.py $n >> $OUT
done
