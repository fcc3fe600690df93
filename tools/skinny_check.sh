# skinny routing: GPU suite, bench line, configs[1]/[4] first packets, first-packet timelines
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/skc_t.log 2>&1
timeout -k 10 500 python bench.py --cpu-baseline 0 > gpurun_out/skc_bench.log 2>&1
timeout -k 10 400 python tools/config_bench.py > gpurun_out/skc_config.log 2>&1
QT_FPG_DUMP=gpurun_out/skc_fpg_cv8.tsv timeout -k 10 300 python tools/first_packet_gaps.py > gpurun_out/skc_fpg_cv8.log 2>&1
QT_FPG_DUMP=gpurun_out/skc_fpg_vc4.tsv QT_FPG_VC=1 QT_FPG_B=4 timeout -k 10 300 python tools/first_packet_gaps.py > gpurun_out/skc_fpg_vc4.log 2>&1
