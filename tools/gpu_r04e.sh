# GPU-box script (r04): per-level channel padding (narrow networks: base 16 / 24 / 48 pad only
# the levels below a multiple of 32) -- narrow + residual tests, the 512x128 bf16 tile tests,
# then ResUNet(16/32/48, 4) benches and the config-4 bf16 A/B benches.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04e}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_res.py "tests/test_gpu_mod.py" -k "narrow or res or rg16_tile_choice or halo or bf16_oracle" \
  > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/$TAG.pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/$TAG.pytest.log | head -30; exit $rc; }
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 4 --warmup 2 --verbose --no-cpu-baseline "$@" \
    > gpurun_out/$TAG.$name.json 2> gpurun_out/$TAG.$name.err
  local rc=$?
  echo "$name rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/$TAG.$name.json')); print(d['value'], d['ms_per_step'], d['roofline']['step_conv_frac'])" 2>/dev/null)"
  return $rc
}
run res16 --config res --base 16 --depth 4 && run res32 --config res --base 32 --depth 4 && \
  run res48 --config res --base 48 --depth 4 && \
  run c4base --config 4 --mfma bf16 && run c4n6 --config 4 --mfma bf16 --opt rg16_n128=6 && \
  run c4n20 --config 4 --mfma bf16 --opt rg16_n128=20 && \
  run c4n20bn --config 4 --mfma bf16 --opt rg16_n128=20 --opt rg16_n128_bn=1
