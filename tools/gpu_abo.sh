# GPU-box script: bench A/B over native schedule options (unet_set_option via --opt), one
# line per arm.  usage: bash tools/gpu_abo.sh TAG "BENCH ARGS" "name=v name=v" "..." ...
# ("-" = the defaults).  Arms run in order in separate processes, each under its own limit.
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; BARGS=$2; shift 2
i=0
for A in "$@"; do
  i=$((i+1))
  OPTS=""
  if [ "$A" != "-" ]; then for kv in $A; do OPTS="$OPTS --opt $kv"; done; fi
  timeout -k 10 300 python bench.py $BARGS --verbose --no-cpu-baseline $OPTS > gpurun_out/$TAG.$i.json 2> gpurun_out/$TAG.$i.err
  rc=$?
  echo "[$A] rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.$i.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['achieved'])" 2>/dev/null)"
  grep -E "^  conv_wgrad |^  conv_dgrad |^  conv_fwd |^  convT" gpurun_out/$TAG.$i.err | head -6
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/$TAG.$i.err; exit $rc; fi
done
