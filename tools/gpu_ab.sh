# GPU-box script: bench A/B over native kernel-schedule options (unet_set_option), with the
# per-kernel / per-layer breakdown in the .err files.
# usage: bash tools/gpu_ab.sh TAG ROUNDS SET1 SET2 ...
#   SETi = comma-separated name=value options ("-" = defaults), e.g. "rg16_tile=0,wg16_tile=0"
#   BENCH_ARGS (env) = extra bench.py arguments, e.g. "--config 4 --mfma bf16 --steps 4"
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; N=$2; shift 2
for r in $(seq 1 $N); do
  i=0
  for S in "$@"; do
    i=$((i+1))
    OPTS=""
    if [ "$S" != "-" ]; then
      for kv in $(echo "$S" | tr ',' ' '); do OPTS="$OPTS --opt $kv"; done
    fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --verbose ${BENCH_ARGS:---steps 10 --warmup 3} $OPTS \
      > gpurun_out/$TAG.r$r.s$i.json 2> gpurun_out/$TAG.r$r.s$i.err
    rc=$?
    echo "round $r set $i [$S] rc=$rc: $(python -c "import json;d=json.load(open('gpurun_out/$TAG.r$r.s$i.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['achieved'])" 2>/dev/null)"
    [ $rc -ne 0 ] && { tail -n 20 gpurun_out/$TAG.r$r.s$i.err; exit $rc; }
  done
done
exit 0
