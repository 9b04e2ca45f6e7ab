# A/B of the multi-workgroup stage: grid size (HGX_CO_BLOCKS), work-item chunk (HGX_CO_CHUNK), barrier
# arrival groups (HGX_CO_BARGROUPS): the per-level trace on config 5's big closures, then the config-5
# bench step (tools/c5_step.py).  OUT=name BLOCKS="..." CHUNKS="..." BARG="..." bash tools/coop_ab.sh
set -e
mkdir -p gpurun_out
log=gpurun_out/${OUT:-coop_ab}.log
for b in ${BLOCKS:-96}; do for c in ${CHUNKS:-128}; do for q in ${BARG:-16}; do
  echo "== blocks $b chunk $c bargroups $q" >> $log
  HGX_CO_TRACE=1 HGX_CO_BLOCKS=$b HGX_CO_CHUNK=$c HGX_CO_BARGROUPS=$q timeout -k 10 120 python -u tools/c5_coop_trace.py >> $log 2>&1
  HGX_CO_BLOCKS=$b HGX_CO_CHUNK=$c HGX_CO_BARGROUPS=$q timeout -k 10 120 python -u tools/c5_step.py --steps 20 >> $log 2>&1
done; done; done
