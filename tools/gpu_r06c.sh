# GPU-box script (r06): config-4 A/B rounds only (tools/gpu_ab.sh), optional pytest -k first.
#   usage: bash tools/gpu_r06c.sh TAG "PYTEST_K" ROUNDS "SET1" "SET2" ...   (PYTEST_K "-" = none)
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; K=$2; N=$3; shift 3
mkdir -p gpurun_out
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -p no:cacheprovider -k "$K" > gpurun_out/$TAG.pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -2
  [ $rc -ne 0 ] && exit $rc
fi
BENCH_ARGS="${C4_ARGS:---config 4 --mfma bf16 --steps 6 --warmup 2}" bash tools/gpu_ab.sh $TAG.c4 $N "$@"
