# GPU-box script (r04): direct-from-global row tiles (15 / 29 / 27 / 28) -- bit-identity tests,
# then A/B benches (narrow ResUNets, config 2 with the 64-output tiles).
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04h}
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_res.py -k "direct_tiles" > gpurun_out/$TAG.pytest.log 2>&1
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
run res32 $R --base 32 && run res32t29 $R --base 32 --opt tile_n32=29 && \
  run res16 $R --base 16 && run res16t29 $R --base 16 --opt tile_n32=29 && \
  run res48 $R --base 48 && run res48n96off $R --base 48 --opt tile_n96=-1 && \
  run res32n64 $R --base 32 --opt tile_n64=27 --opt tile_n64_dgrad=27 && \
  run c2 --steps 10 --warmup 3 && run c2n64 --steps 10 --warmup 3 --opt tile_n64=27 --opt tile_n64_dgrad=27 && \
  run c2n64f --steps 10 --warmup 3 --opt tile_n64=27
