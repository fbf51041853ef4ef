# GPU-box script (r04): the 512x128 bf16 row tiles (one-tap 6, tap-row halo 20) -- their
# bit-identity / bf16-envelope tests, then config-4 bf16 A/B benches (verbose per-kernel tables).
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04d}
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_mod.py::test_rg16_tile_choice_is_numerically_invisible" \
  "tests/test_gpu_mod.py::test_rg16_halo_tile_within_bf16_error" \
  "tests/test_gpu_mod.py::test_mod_bf16_matches_bf16_oracle" \
  > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/$TAG.pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/$TAG.pytest.log | head -30; exit $rc; }
run() {  # name, options...
  local name=$1; shift
  timeout -k 10 300 python bench.py --config 4 --mfma bf16 --steps 4 --warmup 2 --verbose --no-cpu-baseline "$@" \
    > gpurun_out/$TAG.$name.json 2> gpurun_out/$TAG.$name.err
  local rc=$?
  echo "$name rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/$TAG.$name.json')); print(d['value'], d['ms_per_step'], d['roofline']['step_conv_frac'])" 2>/dev/null)"
  return $rc
}
run base && run n6 --opt rg16_n128=6 && run n20 --opt rg16_n128=20 && \
  run n20bn --opt rg16_n128=20 --opt rg16_n128_bn=1 && run base2
