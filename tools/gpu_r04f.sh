# GPU-box script (r04): new bf16 kernels (512x128 row tiles, tap-row weight gradient) and the
# per-level channel padding -- their tests, then benches (narrow ResUNets, config-4 A/B).
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04f}
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_res.py "tests/test_gpu_mod.py" -k "narrow or res or rg16_tile_choice or halo or bf16_oracle or tap_row or convt16 or register_staged or direct_tiles" \
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
run c4base --config 4 --mfma bf16 && run c4r3 --config 4 --mfma bf16 --opt wg16_r3=3 && \
  run c4r4 --config 4 --mfma bf16 --opt wg16_r3=4 && \
  run c4n6 --config 4 --mfma bf16 --opt rg16_n128=6 && \
  run c4n20 --config 4 --mfma bf16 --opt rg16_n128=20 && \
  run c4n20bn --config 4 --mfma bf16 --opt rg16_n128=20 --opt rg16_n128_bn=1 && \
  run res16 --config res --base 16 --depth 4 && run res32 --config res --base 32 --depth 4 && \
  run res48 --config res --base 48 --depth 4 && run res32t15 --config res --base 32 --depth 4 --opt tile_n32=15 && \
  run res32t13 --config res --base 32 --depth 4 --opt tile_n32=13 && run res16t15 --config res --base 16 --depth 4 --opt tile_n32=15 && run c2 --steps 10
