# GPU-box script: the whole -m gpu suite WITHOUT -x (every failure listed), then the config-2
# bench line with CPU baseline.  usage: bash tools/gpu_suite.sh TAG
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-suite}
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider --durations=12 -rP > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -3
grep -E "^FAILED|^ERROR" gpurun_out/$TAG.pytest.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --verbose > gpurun_out/$TAG.c2.json 2> gpurun_out/$TAG.c2.err
rc2=$?
echo "bench rc=$rc2"; cat gpurun_out/$TAG.c2.json | cut -c1-600
exit $rc
