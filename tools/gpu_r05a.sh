# GPU-box script (r05a): x3 numerics tests (masked fp64 bars, range edges, option refusal),
# bench.py's own 2-rank launcher over gloo (DP rehearsal), the bucket timeline + interference
# probe of DESIGN §5, and one verbose config-2 bench.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r05a}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_x3.py > gpurun_out/$TAG.x3.log 2>&1
rc=$?
echo "x3 tests rc=$rc"; grep -E "PASS|FAIL|ERROR|worst|vs fp64|logits" gpurun_out/$TAG.x3.log | tail -40
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --batch 8 \
  > gpurun_out/$TAG.dp2.json 2> gpurun_out/$TAG.dp2.err
rc2=$?
echo "dp2 rc=$rc2"; cat gpurun_out/$TAG.dp2.json; [ $rc2 -ne 0 ] && { tail -30 gpurun_out/$TAG.dp2.err; exit $rc2; }
timeout -k 10 400 python tools/bucket_timeline.py > gpurun_out/$TAG.buckets.json 2> gpurun_out/$TAG.buckets.err
rc3=$?
echo "buckets rc=$rc3"; head -c 3000 gpurun_out/$TAG.buckets.json; [ $rc3 -ne 0 ] && { tail -30 gpurun_out/$TAG.buckets.err; exit $rc3; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose --no-cpu-baseline \
  > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc4=$?
echo "bench rc=$rc4"; cat gpurun_out/$TAG.bench.json; grep -v amdgpu.ids gpurun_out/$TAG.bench.err | head -70
exit $(( rc + rc4 ))
