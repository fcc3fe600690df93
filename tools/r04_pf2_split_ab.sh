# gemm_pf2_k split-K for wide outputs at streaming-prefill sizes: QT_PF2_KS forces the split factor (any shape),
# QT_PF2_CFG the tile; 1.7B talker prefill linears at M = 96 / 160 (B = 8 streaming-text prompts, refill prefills)
set -e
mkdir -p gpurun_out
out=gpurun_out/pf2_split_ab.txt
: > $out
for cfg in 0 3 11; do
  for ks in 0 1 2 4; do
    echo "## cfg=$cfg ks=$ks" >> $out
    QT_PF2_CFG=$cfg QT_PF2_KS=$ks QT_PB_M=96,160 timeout -k 10 120 python tools/prefill_gemm_bench.py >> $out 2>&1
  done
done
