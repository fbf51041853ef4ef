# GPU-box script: mod-variant GPU tests (verbose), then config-4 benches (bf16 and fp32).
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-bf16}
timeout -k 10 600 python -m pytest tests/test_gpu_mod.py -q -s -p no:cacheprovider > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "bf16 base|passed|failed|Error|assert" gpurun_out/$TAG.pytest.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config 4 --mfma bf16 --steps 4 --warmup 2 --verbose --no-cpu-baseline > gpurun_out/$TAG.c4bf16.json 2> gpurun_out/$TAG.c4bf16.err
rc=$?
echo "bench bf16 rc=$rc"; cat gpurun_out/$TAG.c4bf16.json; grep -v amdgpu.ids gpurun_out/$TAG.c4bf16.err | head -45
