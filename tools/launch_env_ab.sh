#!/bin/bash
# Graph launch floor (tools/launch_floor) under HIP runtime environment knobs: grid 256 x block 512 lines only.
# usage (GPU box): bash tools/launch_env_ab.sh > gpurun_out/launch_env_ab.txt
for env in "" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" \
           "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "ROC_SKIP_KERNEL_ARG_COPY=1" "GPU_FLUSH_ON_EXECUTION=0"; do
  echo "== env: ${env:-default}"
  env $env timeout -k 5 60 ./tools/launch_floor > /tmp/lf.txt || { echo "failed $?"; exit 1; }
  awk '/grid   256 x block   512/ || /grid     8 x block   512/' /tmp/lf.txt
done
