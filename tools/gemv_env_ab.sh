#!/bin/bash
# decode GEMV shapes (tools/gemv_hot_cold.py, graphs of 200 launches) under launch-config overrides, one box
# usage: bash tools/gemv_env_ab.sh [VAR=val ...]   (default set below)
set -e
out=gpurun_out/gemv_env_ab.txt
: > $out
cfgs=("$@")
[ ${#cfgs[@]} -eq 0 ] && cfgs=("X=0" "QT_GEMV_WPB=16" "QT_GEMV_WPB=4" "QT_GEMV_RG=2" "QT_GEMV_U=8" "QT_GEMV_RG=1")
for cfg in "${cfgs[@]}"; do
  echo "== $cfg" >> $out
  env $cfg timeout -k 10 200 python tools/gemv_hot_cold.py 2>&1 | grep "us/launch" >> $out
done
