#!/bin/bash
# Profiles the benchmark command with rocprofv3 (run on the GPU box from the repo root):
#   1. kernel trace + stats       -> gpurun_out/prof_<tag>/trace
#   2. PMC FETCH_SIZE (own pass)  -> gpurun_out/prof_<tag>/fetch
#   3. PMC WRITE_SIZE (own pass)  -> gpurun_out/prof_<tag>/write
# Each step runs under its own timeout; the chain stops at the first failure.
set -u
TAG=${1:-r01}
shift || true
ARGS=${@:-"--steps 3 --warmup 1 --no-cpu-baseline"}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py $ARGS \
    > $OUT/trace.json 2> $OUT/trace.log || { echo "trace pass failed $?"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetch -o run -- python3 bench.py $ARGS \
    > $OUT/fetch.json 2> $OUT/fetch.log || { echo "fetch pass failed $?"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/write -o run -- python3 bench.py $ARGS \
    > $OUT/write.json 2> $OUT/write.log || { echo "write pass failed $?"; exit 1; }
echo "profile passes done"
find $OUT -name "*.csv" | head -20
