# GPU-box script: rehearsal of bench.py's N>1 data-parallel path with two ranks on the one
# GPU (gloo instead of RCCL: RCCL refuses two ranks per device).  Checks that the launcher
# contract, the gathered-batch loss all-reduce and the bucketed gradient sum run end to end.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-dp2}
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --batch 8 \
  > gpurun_out/$TAG.json 2> gpurun_out/$TAG.err
rc=$?
echo "dp2 rc=$rc"; cat gpurun_out/$TAG.json; [ $rc -ne 0 ] && tail -30 gpurun_out/$TAG.err
exit $rc
