# talker decode attention with the bf16 v_dot2 consume loop: parity tests, lengths 138..4000 x split factors, bench
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread -k "attention or talker or full_dims or attn_oproj" > gpurun_out/tattn_tests.txt 2>&1
ATTN_L=138,300,512,1024,2048,4000 ATTN_NS=1,2,4,8 timeout -k 10 300 python tools/talker_attn_bench.py > gpurun_out/tattn_long.txt 2>&1
timeout -k 10 600 python bench.py > gpurun_out/bench_tattn.json 2> gpurun_out/bench_tattn.err
