# GPU-box script (r06 round-end evidence): the whole -m gpu suite + the config-2 bench line with
# its CPU baseline (tools/gpu_suite.sh), the config-4 bf16 bench line, smoke(), and the N = 2
# data-parallel rehearsal (two ranks on the one GPU over gloo).   usage: bash tools/gpu_r06final2.sh TAG
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r06final2}
bash tools/gpu_suite.sh $TAG
rc=$?
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --config 4 --mfma bf16 --steps 10 --warmup 3 --verbose --no-cpu-baseline \
  > gpurun_out/$TAG.c4.json 2> gpurun_out/$TAG.c4.err
rc2=$?
echo "c4 bench rc=$rc2"; cut -c1-300 gpurun_out/$TAG.c4.json
[ $rc2 -ne 0 ] && exit $rc2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG.smoke.log 2>&1
rc3=$?
echo "smoke rc=$rc3"; tail -2 gpurun_out/$TAG.smoke.log
[ $rc3 -ne 0 ] && exit $rc3
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/$TAG.dp2.json 2> gpurun_out/$TAG.dp2.err
rc4=$?
echo "dp2 rehearsal rc=$rc4"; grep '^{' gpurun_out/$TAG.dp2.json | cut -c1-300
exit $rc
