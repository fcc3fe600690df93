# GPU suite + bench first packets + first-packet timelines
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fpc_t.log 2>&1
timeout -k 10 500 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/fpc_bench.log 2>&1
QT_FPG_DUMP=gpurun_out/fpc_fpg_cv8.tsv timeout -k 10 300 python tools/first_packet_gaps.py > gpurun_out/fpc_fpg_cv8.log 2>&1
QT_FPG_B=1 timeout -k 10 300 python tools/first_packet_gaps.py > gpurun_out/fpc_fpg_cv1.log 2>&1
