# GPU-box script: a pytest selection (-k expression or file list) with per-test timeouts.
# usage: bash tools/gpu_tests.sh TAG "pytest args..."
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; shift
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|Error" gpurun_out/$TAG.pytest.log | tail -8
exit $rc
