# GPU-box script (r05e): x3 + parity tests, then config-2 bench lines (verbose).
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r05e}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_x3.py tests/test_gpu_parity.py > gpurun_out/$TAG.t.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/$TAG.t.log | tail -8
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose --no-cpu-baseline > gpurun_out/$TAG.b$i.json 2> gpurun_out/$TAG.b$i.err
r=$?
echo "bench rc=$r $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.b$i.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'])" 2>/dev/null)"
[ $r -ne 0 ] && exit $r
done
grep -E "prep_x3|bn_dz|convT_fwd |maxpool_fwd" gpurun_out/$TAG.b1.err
exit 0
