# GPU-box script (r05c): config-4 bf16 schedule A/B (rg16_sched) and the bf16 schedule test.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r05c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_mod.py -k "schedules or wg16_tap_row" > gpurun_out/$TAG.mod.log 2>&1
rc=$?
echo "mod tests rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/$TAG.mod.log | tail -10
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for S in 0 1 2 0; do
  timeout -k 10 300 python bench.py --config 4 --mfma bf16 --steps 8 --warmup 3 --no-cpu-baseline --opt rg16_sched=$S \
    > gpurun_out/$TAG.c4s$S.json 2> gpurun_out/$TAG.c4s$S.err
  r=$?
  echo "rg16_sched $S rc=$r $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.c4s$S.json'));print(d['value'], d['ms_per_step'], d['roofline']['step_conv_frac'])" 2>/dev/null)"
  [ $r -ne 0 ] && { tail -20 gpurun_out/$TAG.c4s$S.err; exit $r; }
done
for S in 5 4; do
  timeout -k 10 300 python bench.py --config 4 --mfma bf16 --steps 8 --warmup 3 --no-cpu-baseline --opt wg16_r3=$S \
    > gpurun_out/$TAG.c4w$S.json 2> gpurun_out/$TAG.c4w$S.err
  r=$?
  echo "wg16_r3 $S rc=$r $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.c4w$S.json'));print(d['value'], d['ms_per_step'], d['roofline']['step_conv_frac'])" 2>/dev/null)"
  [ $r -ne 0 ] && { tail -20 gpurun_out/$TAG.c4w$S.err; exit $r; }
done
exit $rc
