# GPU-box script: bf16 LDS-DMA GEMM tests, then config-4 bf16 bench per rg16 tile (+ register-staged A/B)
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-rg16}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mod.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider -k "${KSEL:-bf16 or rg16}" > gpurun_out/$TAG.pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert|bf16 base" gpurun_out/$TAG.pytest.log | head -30
if [ $rc -ne 0 ]; then tail -30 gpurun_out/$TAG.pytest.log; exit $rc; fi
for T in ${TILES:-}; do
  if [ "$T" = auto ]; then E=""; else E="${TVAR:-UNET_RG16_TILE}=$T"; fi
  env $E timeout -k 10 300 python bench.py --config 4 --mfma bf16 --steps 4 --warmup 2 --verbose --no-cpu-baseline > gpurun_out/$TAG.t$T.json 2> gpurun_out/$TAG.t$T.err
  rc=$?
  echo "tile $T rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/$TAG.t$T.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['achieved'])"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/$TAG.t$T.err; exit $rc; fi
done
grep -v amdgpu.ids gpurun_out/$TAG.t${FIRST:-0}.err | head -40
