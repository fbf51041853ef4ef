# GPU-box script (r06): tests (-k), config-4 / config-2 A/B (tools/gpu_r06d.sh), then the narrow
# ResUNet benches (tools/gpu_r06e.sh).   usage: bash tools/gpu_r06f.sh TAG "PYTEST_K" ROUNDS SETS...
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; K=$2; N=$3; shift 3
bash tools/gpu_r06d.sh $TAG "$K" $N "$@" || exit $?
bash tools/gpu_r06e.sh $TAG.n - "16 24 32 48"
