# GPU-box script: config-4 (bf16) A/B bench lines (no CPU baseline).  usage:
#   bash tools/gpu_c4ab.sh TAG "name1:opts1" "name2:opts2" ...   (opts: space-separated NAME=VALUE)
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; shift
for spec in "$@"; do
  name=${spec%%:*}; opts=${spec#*:}
  args=""; for o in $opts; do args="$args --opt $o"; done
  timeout -k 10 300 python bench.py --config 4 --mfma bf16 --verbose --steps 8 --warmup 2 --no-cpu-baseline $args > gpurun_out/$TAG.$name.json 2> gpurun_out/$TAG.$name.err
  rc=$?
  echo "$name [$opts] rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/$TAG.$name.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['achieved'], r['step_conv_frac'])" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -15 gpurun_out/$TAG.$name.err; exit $rc; }
done
exit 0
