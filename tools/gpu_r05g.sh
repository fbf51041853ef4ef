# GPU-box script (r05g): x3 GPU tests, then a same-box bench A/B of two option settings
#   usage: bash tools/gpu_r05g.sh TAG "TESTS" "OPT_A" "OPT_B" [config]
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r05g}
TESTS=${2:-tests/test_gpu_x3.py}
A=${3:-x3_r3_sched=1}
B=${4:-x3_r3_sched=9}
CFG=${5:-2}
EXTRA=${6:-}
mkdir -p gpurun_out
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    $TESTS > gpurun_out/$TAG.t.log 2>&1
  rc=$?
  echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/$TAG.t.log | tail -6
  [ $rc -ne 0 ] && exit $rc
fi
for O in "$A" "$B" "$A" "$B"; do
  timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline $EXTRA --opt $O > gpurun_out/$TAG.json 2> gpurun_out/$TAG.err
  r=$?
  echo "$O rc=$r $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.json'));print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['kernel'], d['roofline'].get('step_conv_frac'))" 2>/dev/null)"
  [ $r -ne 0 ] && { tail -5 gpurun_out/$TAG.err; exit $r; }
done
exit 0
