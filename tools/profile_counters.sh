#!/bin/bash
# Extra PMC passes (occupancy / LDS / cache counters) of any python command, one rocprofv3 run per pass
# (each within the per-block counter limits), run on the GPU box from the repo root:
#   bash tools/profile_counters.sh <tag> <script.py> [args...]
# -> gpurun_out/prof_<tag>/pmc{1,2,3}/run_counter_collection.csv
set -u
TAG=$1
shift
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY TCC_HIT_sum TCC_MISS_sum"
P3="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TD_BUSY_avr"
i=1
for P in "$P1" "$P2" "$P3"; do
    timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -f csv -d $OUT/pmc$i -o run -- python3 "$@" \
        > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed $?"; exit 1; }
    i=$((i+1))
done
echo "counter passes done: $OUT"
