set -e
P=$GRAFT_REPO_ROOT/qwen3-tts_amd/lib/libqwen3tts_amd_probe.so
for r in 1 2; do
  for pp in 0 1; do
    QWEN3TTS_AMD_LIB=$P QT_PF2_PP=$pp timeout -k 10 200 python tools/pf2_layer_ab.py 256 680 1600 >> gpurun_out/pf2_layer_ab.txt 2>gpurun_out/pf2_layer_ab.err
  done
done
