# GPU-box script: full GPU test suite, config-2 bench (CPU baseline + dice_vs_ref), config-4 bf16 bench.
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-full}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|Error" gpurun_out/$TAG.pytest.log | tail -8
if [ $rc -ne 0 ]; then tail -40 gpurun_out/$TAG.pytest.log; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/$TAG.bench.json; grep -v amdgpu.ids gpurun_out/$TAG.bench.err | head -26
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config 4 --mfma bf16 --steps 4 --warmup 2 --verbose --no-cpu-baseline > gpurun_out/$TAG.c4bf16.json 2> gpurun_out/$TAG.c4bf16.err
rc=$?
echo "bench c4 rc=$rc"; cat gpurun_out/$TAG.c4bf16.json; grep -v amdgpu.ids gpurun_out/$TAG.c4bf16.err | head -34
exit $rc
