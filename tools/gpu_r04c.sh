# GPU-box script (r04): DP of ResUNet / mod.UNet vs the reference DataParallel fixture, the
# narrow (padded) networks with per-bucket compaction, the sped-up full-size tests, then the
# config-4 bf16 bench (verbose per-kernel table).
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04c}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --durations=10 tests/test_gpu_dist.py tests/test_gpu_res.py \
  "tests/test_gpu_mod.py::test_mod_narrow_b32_matches_golden" \
  "tests/test_gpu_mod.py::test_mod_narrow_one_step_matches_golden" \
  "tests/test_gpu_mod.py::test_mod_bf16_matches_bf16_oracle" \
  "tests/test_gpu_parity.py::test_full_size_vs_torch_gpu_reference" \
  > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/$TAG.pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/$TAG.pytest.log | head -30; exit $rc; }
sed -n '/slowest/,$p' gpurun_out/$TAG.pytest.log | head -14
timeout -k 10 400 python bench.py --config 4 --mfma bf16 --steps 4 --warmup 2 --verbose --no-cpu-baseline \
  > gpurun_out/$TAG.c4bf16.json 2> gpurun_out/$TAG.c4bf16.err
rc=$?
echo "bench bf16 rc=$rc"; cat gpurun_out/$TAG.c4bf16.json; grep -v amdgpu.ids gpurun_out/$TAG.c4bf16.err | head -40
exit $rc
