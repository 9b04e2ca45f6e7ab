#!/bin/bash
# rocprofv3 kernel trace + FETCH/WRITE PMC passes of the config-3 pattern batch (run on the GPU box):
#   bash tools/profile_pattern.sh <tag>   ->  gpurun_out/prof_<tag>/{trace,fetch,write}
set -u
TAG=${1:-r01q}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
CMD="python3 tools/pattern_timing.py --calls 6"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- $CMD > $OUT/trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1 || { echo "write pass failed"; exit 1; }
echo "pattern profile passes done"
