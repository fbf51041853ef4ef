# GPU-box script: rocprofv3 kernel-trace stats + PMC passes (HBM bytes, MFMA busy) of both
# bench workloads: config 2 (fp32) and config 4 (bf16).  Outputs under gpurun_out/TAG.*
set -u
R=$GRAFT_REPO_ROOT
TAG=${1:-prof}
cd /tmp && export TMPDIR=/tmp
for C in ${CONFIGS:-c2 c4}; do
  if [ $C = c2 ]; then ARGS="--steps 3 --warmup 1 --no-cpu-baseline"; else ARGS="--config 4 --mfma bf16 --steps 2 --warmup 1 --no-cpu-baseline"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG.$C.prof -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/$TAG.$C.prof.log 2>&1
  rc=$?
  echo "$C rocprof rc=$rc"; tail -1 $R/gpurun_out/$TAG.$C.prof.log | cut -c1-300
  if [ $rc -ne 0 ]; then tail -20 $R/gpurun_out/$TAG.$C.prof.log; exit $rc; fi
  head -8 $R/gpurun_out/$TAG.$C.prof/run_kernel_stats.csv | cut -c1-200
  i=0
  for CN in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $CN --output-format csv -d $R/gpurun_out/$TAG.$C.pmc$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/$TAG.$C.pmc$i.log 2>&1
    rc=$?
    echo "$C pmc pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/$TAG.$C.pmc$i.log; exit $rc; fi
  done
  (cd $R && python3 tools/pmc_summary.py gpurun_out/$TAG.pmc_summary_$C.json gpurun_out/$TAG.$C.pmc1 gpurun_out/$TAG.$C.pmc2 gpurun_out/$TAG.$C.pmc3)
done
