# Round-4 probe 5: decode attention with a 4-deep register-set ring for split (long-cache) launches.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "decode_attention or split_kv or attn_oproj" > gpurun_out/r04_t_attn_ring.txt 2>&1
ATTN_L=138,512,1024,2048,4000 ATTN_NS=1,2,4,8 timeout -k 10 300 python tools/talker_attn_bench.py > gpurun_out/r04_attn_ring_default.txt 2>&1
QT_ATTN_NB=4 ATTN_L=138,300,512,1024 ATTN_NS=1 timeout -k 10 200 python tools/talker_attn_bench.py > gpurun_out/r04_attn_ring_nb4_ns1.txt 2>&1
