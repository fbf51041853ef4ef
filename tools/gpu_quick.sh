# GPU-box script: config-2 bench (with CPU baseline + dice_vs_ref), then config-4 bf16 bench, verbose.
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-quick}
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/$TAG.bench.json; grep -v amdgpu.ids gpurun_out/$TAG.bench.err | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${2:-}" = "c4" ]; then
timeout -k 10 400 python bench.py --config 4 --mfma bf16 --steps 4 --warmup 2 --verbose --no-cpu-baseline > gpurun_out/$TAG.c4bf16.json 2> gpurun_out/$TAG.c4bf16.err
rc=$?
echo "bench bf16 rc=$rc"; cat gpurun_out/$TAG.c4bf16.json; grep -v amdgpu.ids gpurun_out/$TAG.c4bf16.err | head -70
fi
exit $rc
