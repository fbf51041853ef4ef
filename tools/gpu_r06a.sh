# GPU-box script (r06): baseline per-layer tables of config 4 (bf16) and config 2 on one box.
#   usage: bash tools/gpu_r06a.sh TAG
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r06a}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 4 --mfma bf16 --verbose --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG.c4.json 2> gpurun_out/$TAG.c4.err
r=$?; echo "c4 rc=$r"; cut -c1-300 gpurun_out/$TAG.c4.json; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python bench.py --verbose --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG.c2.json 2> gpurun_out/$TAG.c2.err
r=$?; echo "c2 rc=$r"; cut -c1-300 gpurun_out/$TAG.c2.json
exit $r
