# decode kernel table (per-launch us at production shapes) under the library's GEMV knobs, one process per setting
set -e
mkdir -p gpurun_out
out=gpurun_out/gemv_knobs.txt
: > $out
run() { env "$@" KT_TAG="$*" timeout -k 10 240 python tools/kernel_table.py 2>/dev/null | tail -1 >> $out; }
run QT_NONE=0
run QT_GEMV_U=8
run QT_GEMV_FOLD=2
run QT_GEMV_FOLD=1
run QT_GEMV_WPB=4
run QT_GEMV_WPB=8
run QT_GEMV_WPB=16
run QT_GEMV_NT=0
run QT_GEMV_NT=1
run QT_GEMV_SPLIT_AUTO=1
run QT_GEMV_SPLIT_AUTO=4
run QT_NONE=1
