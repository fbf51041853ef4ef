# GPU-box script (r04): the whole -m gpu suite (timed per test), then the config-2 bench.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04b}
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=25 > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -5
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/$TAG.pytest.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/$TAG.bench.json
exit $rc
