# voxel-conv weight-gradient A/B (dev): bash tools/wg_dec.sh <variant names...>
# (variants built by `make variant NAME=... DEFS=...`; the round-5 decomposition
# macros and the one-wave form are in commit 10d43e1)
set -e
V=point-cloud-flow-matching_amd/csrc/build/variants
OUT=gpurun_out/wg_dec.jsonl
timeout -k 10 120 python tools/conv_ab.py main > $OUT
for n in "$@"; do
  PCFM_LIB=$V/libpcfm_$n.so timeout -k 10 120 python tools/conv_ab.py $n >> $OUT
done
