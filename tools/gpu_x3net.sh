# GPU-box script: the config-2 network on the x3 kernels -- parity tests, then bench lines
# with x3 on (default) and off.  usage: bash tools/gpu_x3net.sh TAG [pytest selection]
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-x3n}
SEL=${2:-tests/test_gpu_parity.py}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider --durations=10 > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert|^E " gpurun_out/$TAG.pytest.log | head -40; exit $rc; }
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --verbose "$@" > gpurun_out/$TAG.$name.json 2> gpurun_out/$TAG.$name.err
  local rc=$?
  echo "$name rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/$TAG.$name.json')); print(d['value'], d['ms_per_step'], d['roofline']['step_conv_frac'])" 2>/dev/null)"
  [ $rc -ne 0 ] && tail -15 gpurun_out/$TAG.$name.err
  return $rc
}
run c2x3 --steps 20 --warmup 3 --no-cpu-baseline && run c2f32 --steps 20 --warmup 3 --no-cpu-baseline --opt x3=0 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG.c2x3.err | head -40
