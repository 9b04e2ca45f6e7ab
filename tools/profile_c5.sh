#!/bin/bash
# rocprofv3 kernel trace of the config-5 bench step (tools/c5_step.py, both directions side by side;
# run on the GPU box):  bash tools/profile_c5.sh <tag>   ->  gpurun_out/prof_<tag>/trace (csv + stats)
set -u
TAG=${1:-c5}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 tools/c5_step.py --mode concurrent --steps 20 \
    > $OUT/trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
echo "config-5 trace done"
