# GPU-box script (r06 evidence): the whole -m gpu suite + the config-2 bench line with its CPU
# baseline (tools/gpu_suite.sh), then the config-4 bf16 bench line.   usage: bash tools/gpu_r06final.sh TAG
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r06final}
bash tools/gpu_suite.sh $TAG
rc=$?
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --config 4 --mfma bf16 --steps 10 --warmup 3 --verbose --no-cpu-baseline \
  > gpurun_out/$TAG.c4.json 2> gpurun_out/$TAG.c4.err
rc2=$?
echo "c4 bench rc=$rc2"; cut -c1-400 gpurun_out/$TAG.c4.json
exit $rc
