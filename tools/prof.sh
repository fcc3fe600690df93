#!/bin/bash
# usage: prof.sh <tag> <bench args...>
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 bench.py "$@" > gpurun_out/$tag.log 2>&1
rc=$?
echo rc=$rc >> gpurun_out/$tag.log
find gpurun_out/$tag -name "*kernel_trace*" -delete
exit $rc
