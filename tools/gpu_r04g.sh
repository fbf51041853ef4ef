# GPU-box script (r04): the whole -m gpu suite on the new defaults (tile 15, rg16_n128 20,
# wg16_r3 4, convt16), then config-2 / config-4 / narrow ResUNet benches.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04g}
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=15 > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/$TAG.pytest.log | head -30; exit $rc; }
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --verbose "$@" > gpurun_out/$TAG.$name.json 2> gpurun_out/$TAG.$name.err
  local rc=$?
  echo "$name rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/$TAG.$name.json')); print(d['value'], d['ms_per_step'], d['roofline']['step_conv_frac'])" 2>/dev/null)"
  return $rc
}
run c2 --steps 20 --warmup 3 && run c4 --config 4 --mfma bf16 --steps 6 --warmup 2 --no-cpu-baseline && \
  run res16 --config res --base 16 --depth 4 --steps 6 --warmup 2 --no-cpu-baseline && \
  run res32 --config res --base 32 --depth 4 --steps 6 --warmup 2 --no-cpu-baseline && \
  run res48 --config res --base 48 --depth 4 --steps 6 --warmup 2 --no-cpu-baseline
