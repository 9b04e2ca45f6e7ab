#!/bin/bash
# rocprofv3 passes of any python command (run on the GPU box from the repo root):
#   bash tools/profile_cmd.sh <tag> <script.py> [args...]
#   1. kernel trace + stats       -> gpurun_out/prof_<tag>/trace
#   2. PMC FETCH_SIZE (own pass)  -> gpurun_out/prof_<tag>/fetch
#   3. PMC WRITE_SIZE (own pass)  -> gpurun_out/prof_<tag>/write
# then, in this container: python tools/pmc_summary.py gpurun_out/prof_<tag> <tag> <workload>.
# Each pass runs under its own timeout; the chain stops at the first failure.
set -u
TAG=$1
shift
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 "$@" \
    > $OUT/trace.log 2>&1 || { echo "trace pass failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetch -o run -- python3 "$@" \
    > $OUT/fetch.log 2>&1 || { echo "fetch pass failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/write -o run -- python3 "$@" \
    > $OUT/write.log 2>&1 || { echo "write pass failed $?"; exit 1; }
echo "profile passes done: $OUT"
