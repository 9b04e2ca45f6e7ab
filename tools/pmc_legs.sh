#!/bin/bash
# Counter passes behind every roofline object of the bench line, one rocprofv3 run per pass and leg (run on
# the GPU box from the repo root), then in this container:
#   python tools/pmc_summary.py gpurun_out/prof_<tag>_c2  <tag>_c2  config2
#   python tools/pmc_summary.py gpurun_out/prof_<tag>_c3  <tag>_c3  config3
#   python tools/pmc_summary.py gpurun_out/prof_<tag>_d2  <tag>_d2  dropin2 --from-last hgx_ls_seed
#   python tools/pmc_summary.py gpurun_out/prof_<tag>_d5a <tag>_d5a dropin5_subsumed
#   python tools/pmc_summary.py gpurun_out/prof_<tag>_d5b <tag>_d5b dropin5_subsumes
#   python tools/pmc_summary.py gpurun_out/prof_<tag>_c5  <tag>_c5  config5
#   bash tools/pmc_legs.sh <tag> [legs...]     (legs: c2 c3 c5 d2 d5a d5b; default all)
# Each pass runs under its own timeout; the chain stops at the first failure.
set -u
TAG=$1
shift
LEGS=${@:-"c2 c3 c5 d2 d5a d5b"}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for L in $LEGS; do
    case $L in
        c2) CMD="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-queries --no-config4 --no-config5 --no-dropin" ;;
        c3) CMD="tools/pattern_timing.py --calls 6" ;;
        c5) CMD="tools/c5_step.py --mode concurrent --steps 20" ;;
        d2) CMD="tools/seq_c2.py --reps 2" ;;
        d5a) CMD="tools/seq_c5.py --engines 0 --single 0 --reps 5 --direction subsumed" ;;
        d5b) CMD="tools/seq_c5.py --engines 0 --single 0 --reps 5 --direction subsumes" ;;
        *) echo "unknown leg $L"; exit 2 ;;
    esac
    OUT=gpurun_out/prof_${TAG}_$L
    mkdir -p $OUT
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $CMD \
        > $OUT/trace.log 2>&1 || { echo "$L trace pass failed $?"; exit 1; }
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetch -o run -- python3 $CMD \
        > $OUT/fetch.log 2>&1 || { echo "$L fetch pass failed $?"; exit 1; }
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/write -o run -- python3 $CMD \
        > $OUT/write.log 2>&1 || { echo "$L write pass failed $?"; exit 1; }
    echo "$L passes done: $OUT"
done
