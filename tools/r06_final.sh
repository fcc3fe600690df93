# Round-6 final measurement set (run through gpurun from the repo root) on the final build: tools/r06_prof.sh (bench
# line, rocprof kernel stats, PMC passes), the BASELINE configs[1] / [4] config bench with the configs[4] first-packet
# trace, and the prefill-linear layer A/B (probe library, QT_PF2_PP=0/1) at M = 4096.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
bash tools/r06_prof.sh
cd $R
timeout -k 10 400 python tools/config_bench.py --configs 1 4 > gpurun_out/r06_config_bench.jsonl 2>gpurun_out/r06_config_bench.err
QT_FPG_VC=1 QT_FPG_B=4 timeout -k 10 300 python tools/first_packet_gaps.py > gpurun_out/r06_fpg_vc4.txt 2>&1
P=$R/qwen3-tts_amd/lib/libqwen3tts_amd_probe.so
for pp in 0 1; do
  QWEN3TTS_AMD_LIB=$P QT_PF2_PP=$pp timeout -k 10 300 python tools/pf2_layer_ab.py 680 4096 >> gpurun_out/pf2_layer_ab_4096.txt 2>>gpurun_out/pf2_layer_ab.err
done
echo done
