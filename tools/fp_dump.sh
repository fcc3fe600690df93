set -e
QT_FPG_DUMP=gpurun_out/fpd_cv8.tsv timeout -k 10 300 python tools/first_packet_gaps.py > gpurun_out/fpd_cv8.log 2>&1
timeout -k 10 400 python tools/config_bench.py > gpurun_out/fpd_config.log 2>&1
