# GPU-box script (r05d): x3 for the 32-channel layers (option x3_n32): parity tests, then ResUNet
# narrow-width bench lines with and without it.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r05d}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_mod.py tests/test_gpu_res.py -k "full_grads" > gpurun_out/$TAG.n32.log 2>&1
rc=$?
echo "n32 tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/$TAG.n32.log | tail -30
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for B in ${BASES:-16 24 32 48}; do
  for N in 1 0; do
    timeout -k 10 300 python bench.py --config res --base $B --depth 4 --steps 6 --warmup 2 --opt x3_n32=$N \
      > gpurun_out/$TAG.res${B}n$N.json 2> gpurun_out/$TAG.res${B}n$N.err
    r=$?
    echo "res base $B x3_n32 $N rc=$r $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.res${B}n$N.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['kernel'], r.get('step_conv_fp32_mfma_frac'), r['step_conv_frac'])" 2>/dev/null)"
    [ $r -ne 0 ] && { tail -20 gpurun_out/$TAG.res${B}n$N.err; exit $r; }
  done
done
exit $rc
