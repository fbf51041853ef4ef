# GPU-box script (r06): narrow-width GPU tests (-k, "-" = none), then the reference grid's
# ResUNet(base, 4) benches at 512^2 (bench.py --config res).
#   usage: bash tools/gpu_r06e.sh TAG "PYTEST_K" "BASES"
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; K=$2; BASES=${3:-16 24 32 48}
mkdir -p gpurun_out
if [ "$K" != "-" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -p no:cacheprovider -k "$K" > gpurun_out/$TAG.pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -2
  grep -E "^FAILED|^ERROR" gpurun_out/$TAG.pytest.log | head
  [ $rc -ne 0 ] && exit $rc
fi
for B in $BASES; do
  timeout -k 10 300 python bench.py --config res --base $B --depth 4 --no-cpu-baseline --verbose --steps 10 --warmup 3 \
    > gpurun_out/$TAG.res$B.json 2> gpurun_out/$TAG.res$B.err
  rc=$?
  echo "res base $B rc=$rc: $(python -c "import json;d=json.load(open('gpurun_out/$TAG.res$B.json'));print(d['value'],d['ms_per_step'],d['roofline'].get('step_conv_frac'))" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -n 20 gpurun_out/$TAG.res$B.err; exit $rc; }
done
exit 0
