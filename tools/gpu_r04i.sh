# GPU-box script (r04): 32-channel row3 weight gradients (tiles 24..26) -- narrow-network
# parity tests, then res benches with the option on / off.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04i}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_res.py "tests/test_gpu_mod.py" -k "narrow or res_ or direct_tiles" > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/$TAG.pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/$TAG.pytest.log | head -30; exit $rc; }
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --verbose --no-cpu-baseline "$@" > gpurun_out/$TAG.$name.json 2> gpurun_out/$TAG.$name.err
  local rc=$?
  echo "$name rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/$TAG.$name.json')); print(d['value'], d['ms_per_step'], d['roofline']['step_conv_frac'])" 2>/dev/null)"
  return $rc
}
R="--config res --depth 4 --steps 5 --warmup 2"
run res32 $R --base 32 && run res32off $R --base 32 --opt wgrad_row3_n32=0 && \
  run res16 $R --base 16 && run res16off $R --base 16 --opt wgrad_row3_n32=0 && \
  run res32b $R --base 32
