# GPU-box script (r06): the whole -m gpu suite + config-2 bench line (tools/gpu_suite.sh), then
# config-4 A/B rounds over option sets (tools/gpu_ab.sh).  Test failures (pytest rc 1) do not
# stop the A/B; a crash, abort or timeout does.
#   usage: bash tools/gpu_r06b.sh TAG ROUNDS "SET1" "SET2" ...
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; N=$2; shift 2
mkdir -p gpurun_out
bash tools/gpu_suite.sh $TAG
rc=$?
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
[ "$N" = "0" ] && exit $rc
BENCH_ARGS="--config 4 --mfma bf16 --steps 6 --warmup 2" bash tools/gpu_ab.sh $TAG.c4 $N "$@" || exit $?
exit $rc
