# GPU-box script (r06): selected GPU tests (-k EXPR), then A/B bench rounds of config 4 (bf16)
# and config 2 over option sets.
#   usage: bash tools/gpu_r06t.sh TAG "PYTEST_K" ROUNDS "SET1" "SET2" ...   (SET: a,b=c or "-")
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; K=$2; N=$3; shift 3
mkdir -p gpurun_out
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -p no:cacheprovider -k "$K" > gpurun_out/$TAG.pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -2
  grep -E "^FAILED|^ERROR|Error" gpurun_out/$TAG.pytest.log | head -20
  [ $rc -ne 0 ] && exit $rc
fi
[ "$N" = "0" ] && exit 0
BENCH_ARGS="--config 4 --mfma bf16 --steps 6 --warmup 2" bash tools/gpu_ab.sh $TAG.c4 $N "$@" || exit $?
BENCH_ARGS="--steps 10 --warmup 3" bash tools/gpu_ab.sh $TAG.c2 $N "$@"
