# GPU-box script (r05 final): the whole -m gpu suite, the default config-2 bench line (with the
# CPU baseline), a --verbose family breakdown, then the default config-4 bf16 line.
#   usage: bash tools/gpu_r05final.sh TAG
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r05final}
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider --durations=12 -rP > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -2
grep -E "^FAILED|^ERROR" gpurun_out/$TAG.pytest.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/$TAG.c2.json 2> gpurun_out/$TAG.c2.err
r=$?; echo "bench rc=$r"; cut -c1-400 gpurun_out/$TAG.c2.json; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verbose --no-cpu-baseline > gpurun_out/$TAG.v.json 2> gpurun_out/$TAG.v.err
r=$?; echo "verbose rc=$r"; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python bench.py --config 4 --mfma bf16 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG.c4.json 2> gpurun_out/$TAG.c4.err
r=$?; echo "c4 rc=$r"; cut -c1-300 gpurun_out/$TAG.c4.json
exit $rc
