# GPU-box script (r04, re-entry): the whole -m gpu suite, then the bench lines (config 2 with
# CPU baseline, config 4 bf16, narrow ResUNets at depth 4, 512²).  Outputs under gpurun_out/TAG.*
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04k}
SUITE=${SUITE:-1}
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --verbose "$@" > gpurun_out/$TAG.$name.json 2> gpurun_out/$TAG.$name.err
  local rc=$?
  echo "$name rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/$TAG.$name.json')); print(d['value'], d['ms_per_step'], d['roofline']['step_conv_frac'])" 2>/dev/null)"
  [ $rc -ne 0 ] && tail -15 gpurun_out/$TAG.$name.err
  return $rc
}
if [ $SUITE = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -p no:cacheprovider --durations=15 > gpurun_out/$TAG.pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -3
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/$TAG.pytest.log | head -30; exit $rc; }
fi
R="--config res --depth 4 --steps 5 --warmup 2 --no-cpu-baseline"
run c2 --steps 20 --warmup 3 && run c4 --config 4 --mfma bf16 --steps 6 --warmup 2 --no-cpu-baseline && \
  run res32 $R --base 32 && run res16 $R --base 16 && run res48 $R --base 48 && run res24 $R --base 24 || exit 1
