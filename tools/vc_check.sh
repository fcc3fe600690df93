set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/vcc_t.log 2>&1
timeout -k 10 400 python tools/config_bench.py --configs 4 > gpurun_out/vcc_config.log 2>&1
QT_FPG_DUMP=gpurun_out/vcc_fpg_vc4.tsv QT_FPG_VC=1 QT_FPG_B=4 timeout -k 10 300 python tools/first_packet_gaps.py > gpurun_out/vcc_fpg_vc4.log 2>&1
