# GPU-box script (r04): A/B of the 32-channel row3 weight gradient, then the whole -m gpu suite,
# the bench lines (config 2 with CPU baseline, config 4 bf16, narrow ResUNets) and the rocprofv3
# kernel-trace + PMC passes of configs 2 and 4.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04j}
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --verbose "$@" > gpurun_out/$TAG.$name.json 2> gpurun_out/$TAG.$name.err
  local rc=$?
  echo "$name rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/$TAG.$name.json')); print(d['value'], d['ms_per_step'], d['roofline']['step_conv_frac'])" 2>/dev/null)"
  return $rc
}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/wbw.hip -o /tmp/wbw 2>/dev/null && \
  timeout -k 10 60 /tmp/wbw > gpurun_out/$TAG.wbw.txt 2>&1; cat gpurun_out/$TAG.wbw.txt
R="--config res --depth 4 --steps 5 --warmup 2 --no-cpu-baseline"
run res32 $R --base 32 && run res32off $R --base 32 --opt wgrad_row3_n32=0 && \
  run res32dz0 $R --base 32 --opt dz_in_wgrad=0 && \
  run res16 $R --base 16 && run res16off $R --base 16 --opt wgrad_row3_n32=0 || exit 1
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=15 > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/$TAG.pytest.log | head -30; exit $rc; }
run c2 --steps 20 --warmup 3 && run c4 --config 4 --mfma bf16 --steps 6 --warmup 2 --no-cpu-baseline && \
  run res48 $R --base 48 && run res24 $R --base 24 || exit 1
CONFIGS="c2 c4" bash tools/gpu_prof.sh $TAG
