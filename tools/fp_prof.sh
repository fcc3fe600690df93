# first-packet GPU timelines (torch.profiler): configs[2] B=8 stream and configs[4] voice clone (B=4 per GPU)
set -e
QT_FPG_DUMP=gpurun_out/fpg_cv8.tsv timeout -k 10 300 python tools/first_packet_gaps.py > gpurun_out/fpg_cv8.log 2>&1
QT_FPG_DUMP=gpurun_out/fpg_vc4.tsv QT_FPG_VC=1 QT_FPG_B=4 timeout -k 10 300 python tools/first_packet_gaps.py > gpurun_out/fpg_vc4.log 2>&1
