# GPU-box script: a pytest selection (KSEL over tests/ -m gpu) then both benches
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-q2}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "${KSEL:-adamw}" > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|Error" gpurun_out/$TAG.pytest.log | tail -5
if [ $rc -ne 0 ]; then tail -40 gpurun_out/$TAG.pytest.log; exit $rc; fi
bash tools/gpu_bench2.sh $TAG
