#!/bin/bash
# usage (GPU box, repo root): bash tools/gemv_ab.sh -> gpurun_out/gemv_ab.jsonl (one line per variant)
out=gpurun_out/gemv_ab.jsonl
: > $out
for cfg in "" "QT_GEMV_U=8" "QT_GEMV_U=4"; do
  env $cfg timeout -k 10 300 python3 tools/gemv_ab.py >> $out 2>> gpurun_out/gemv_ab.err || exit 1
done
