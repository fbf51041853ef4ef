# GPU-box script (r05b): halo x3 GEMM schedules (library X3R3Sched + harness flags), the x3
# GPU tests, then config-2 bench lines per x3_r3_sched.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r05b}
FL=${2:-0,96,4096,4160,7}
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3_halo_exp.hip -o /tmp/x3_halo_exp > gpurun_out/$TAG.build.log 2>&1 || { tail -20 gpurun_out/$TAG.build.log; exit 1; }
timeout -k 10 300 /tmp/x3_halo_exp 10 $FL > gpurun_out/$TAG.halo.txt 2>&1
rc=$?
cat gpurun_out/$TAG.halo.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_x3.py > gpurun_out/$TAG.x3.log 2>&1
rc=$?
echo "x3 tests rc=$rc"; grep -E "PASS|FAIL|ERROR|worst|vs fp64|logits|Error" gpurun_out/$TAG.x3.log | tail -40
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for S in 0 1 2 3 4 0; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --opt x3_r3_sched=$S \
    > gpurun_out/$TAG.bench$S.json 2> gpurun_out/$TAG.bench$S.err
  r=$?
  echo "sched $S rc=$r $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.bench$S.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])" 2>/dev/null)"
  [ $r -ne 0 ] && { tail -20 gpurun_out/$TAG.bench$S.err; exit $r; }
done
for S in 6 5; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --opt x3_n64_r3=$S \
    > gpurun_out/$TAG.nbench$S.json 2> gpurun_out/$TAG.nbench$S.err
  r=$?
  echo "n64_r3 $S rc=$r $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.nbench$S.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  [ $r -ne 0 ] && { tail -20 gpurun_out/$TAG.nbench$S.err; exit $r; }
done
for S in ${WS:-1 2 0}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --opt x3_wsched=$S \
    > gpurun_out/$TAG.wbench$S.json 2> gpurun_out/$TAG.wbench$S.err
  r=$?
  echo "wsched $S rc=$r $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.wbench$S.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  [ $r -ne 0 ] && { tail -20 gpurun_out/$TAG.wbench$S.err; exit $r; }
done
exit $rc
