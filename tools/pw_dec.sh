# pointwise GEMM decomposition A/B (dev): bash tools/pw_dec.sh <variant names...>
set -e
V=point-cloud-flow-matching_amd/csrc/build/variants
OUT=gpurun_out/pw_dec.jsonl
PCFM_PW_GLDS=0 timeout -k 10 120 python tools/pw_ab.py staged > $OUT
timeout -k 10 120 python tools/pw_ab.py glds >> $OUT
for n in "$@"; do
  PCFM_LIB=$V/libpcfm_$n.so timeout -k 10 120 python tools/pw_ab.py $n >> $OUT
done
