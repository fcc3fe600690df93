# talker decode attention, bf16 v_dot2 loop: 8 vs 16 waves per (row, kv head) block (QT_ATTN_NW16), parity + lengths
set -e
mkdir -p gpurun_out
QT_ATTN_NW16=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 150 --timeout-method thread -k "decode_attention or split_kv" > gpurun_out/nw16_tests.txt 2>&1
for nw in 0 1; do
  QT_ATTN_NW16=$nw ATTN_L=138,267,460,1024,2048 ATTN_NS=1,2,4 timeout -k 10 300 python tools/talker_attn_bench.py > gpurun_out/nw16_$nw.txt 2>&1
done
