set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/attn_ep_t.log 2>&1
QT_ATTN_EP=0 ATTN_NS=1 timeout -k 10 300 python tools/talker_attn_bench.py > gpurun_out/attn_ep0.log 2>&1
QT_ATTN_EP=1 ATTN_NS=1 timeout -k 10 300 python tools/talker_attn_bench.py > gpurun_out/attn_ep1.log 2>&1
QT_ATTN_EP=0 timeout -k 10 400 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/attn_bench0.log 2>&1
QT_ATTN_EP=1 timeout -k 10 400 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/attn_bench1.log 2>&1
