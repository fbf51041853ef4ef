# GPU-box script: tests, then bench, then an optional rocprofv3 kernel-trace pass.
# usage: bash tools/gpu_run.sh TAG [prof]
set -u
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/$TAG.pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/$TAG.bench.json; grep -v amdgpu.ids gpurun_out/$TAG.bench.err | head -40
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${2:-}" = "prof" ] || [ "${3:-}" = "prof" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG.prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/$TAG.prof.log 2>&1
  echo "rocprof rc=$?"
  head -12 $R/gpurun_out/$TAG.prof/run_kernel_stats.csv | cut -c1-160
fi
if [ "${2:-}" = "pmc" ] || [ "${3:-}" = "pmc" ]; then
  cd /tmp && export TMPDIR=/tmp
  i=0
  for CN in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $CN --output-format csv -d $R/gpurun_out/$TAG.pmc$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/$TAG.pmc$i.log 2>&1
    rc=$?
    echo "pmc pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/$TAG.pmc$i.log; exit $rc; fi
  done
  cd $R && python3 tools/pmc_summary.py gpurun_out/$TAG.pmc_summary.json gpurun_out/$TAG.pmc1 gpurun_out/$TAG.pmc2 gpurun_out/$TAG.pmc3
fi
