# tools/pf2_layer_ab.py A/B on one box: the probe library with QT_PF2_PP=0 (ping-pong configurations left out of the
# picker) and 1 (product), two rounds, at the M values given (default 256 680 1600).
set -e
P=$GRAFT_REPO_ROOT/qwen3-tts_amd/lib/libqwen3tts_amd_probe.so
Ms=${*:-256 680 1600}
for r in 1 2; do
  for pp in 0 1; do
    QWEN3TTS_AMD_LIB=$P QT_PF2_PP=$pp timeout -k 10 300 python tools/pf2_layer_ab.py $Ms >> gpurun_out/pf2_layer_ab.txt 2>gpurun_out/pf2_layer_ab.err
  done
done
