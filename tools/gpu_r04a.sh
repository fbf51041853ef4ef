# GPU-box script (r04): bench.py's own N-rank launcher rehearsed with gloo on the one GPU,
# the 2-rank Trainer hygiene test, then the config-4 bf16 bench (verbose per-kernel table).
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04a}
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --batch 8 \
  > gpurun_out/$TAG.dp2.json 2> gpurun_out/$TAG.dp2.err
rc=$?
echo "dp2 rc=$rc"; cat gpurun_out/$TAG.dp2.json; [ $rc -ne 0 ] && { tail -30 gpurun_out/$TAG.dp2.err; exit $rc; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dist.py -k hygiene > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/$TAG.pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --config 4 --mfma bf16 --steps 4 --warmup 2 --verbose --no-cpu-baseline \
  > gpurun_out/$TAG.c4bf16.json 2> gpurun_out/$TAG.c4bf16.err
rc=$?
echo "bench bf16 rc=$rc"; cat gpurun_out/$TAG.c4bf16.json; grep -v amdgpu.ids gpurun_out/$TAG.c4bf16.err | head -60
exit $rc
