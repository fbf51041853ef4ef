# GPU-box script (r05f): x3 weight-gradient schedule 3 (late DMA): bit-identity test + bench A/B
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r05f}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_x3.py -k "wgrad_schedules" > gpurun_out/$TAG.t.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/$TAG.t.log | tail -4
[ $rc -ne 0 ] && exit $rc
for S in 3 0 3 0; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --opt x3_wsched=$S > gpurun_out/$TAG.w$S.json 2> gpurun_out/$TAG.w$S.err
  r=$?
  echo "wsched $S rc=$r $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.w$S.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  [ $r -ne 0 ] && exit $r
done
exit 0
