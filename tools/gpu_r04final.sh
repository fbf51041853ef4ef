# GPU-box script (r04 close): smoke(), the narrow / residual ResUNet bench lines on the final
# kernels (x3 where channels allow) and the config-4 bf16 bench line.  usage: bash tools/gpu_r04final.sh TAG
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r04z}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG.smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/$TAG.smoke.log)"; [ $rc -ne 0 ] && exit $rc
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline "$@" \
    > gpurun_out/$TAG.$name.json 2> gpurun_out/$TAG.$name.err
  local rc=$?
  echo "$name rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/$TAG.$name.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['step_conv_frac'], r.get('step_conv_fp32_mfma_frac'))" 2>/dev/null)"
  return $rc
}
run res16 --config res --base 16 --depth 4 && run res24 --config res --base 24 --depth 4 && \
  run res32 --config res --base 32 --depth 4 && run res48 --config res --base 48 --depth 4 && \
  run res64 --config res --base 64 --depth 4 && run c4 --config 4 --mfma bf16
