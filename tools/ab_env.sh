#!/bin/bash
# Kernel traces of one command under several environment settings (A/B of engine knobs; the knobs are read
# only by A/B builds: bash tools/build_variant.sh ab, then HGX_LIB_VARIANT=ab in the settings), run on the
# GPU box from the repo root:
#   bash tools/ab_env.sh <tag> "<VAR=v VAR2=w>" "<VAR=x>" ... -- <script.py> [args...]
# Each setting gets gpurun_out/ab_<tag>/<k>/ (rocprofv3 --kernel-trace --stats) and a line in
# gpurun_out/ab_<tag>/settings.txt; summarise with python tools/ab_summary.py gpurun_out/ab_<tag>.
# Every pass runs under its own timeout; the chain stops at the first failure.
set -u
TAG=$1
shift
SETTINGS=()
while [ "$#" -gt 0 ] && [ "$1" != "--" ]; do SETTINGS+=("$1"); shift; done
shift
OUT=gpurun_out/ab_${TAG}
mkdir -p $OUT
: > $OUT/settings.txt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
k=0
for S in "${SETTINGS[@]}"; do
    echo "$k $S" >> $OUT/settings.txt
    (
        for kv in $S; do export "$kv"; done
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/$k -o run -- python3 "$@" > $OUT/$k.log 2>&1
    ) || { echo "setting $k failed"; exit 1; }
    k=$((k + 1))
done
echo "ab passes done: $OUT"
