# GPU-box script (r06): selected GPU tests (-k, "-" = none), then bench A/B rounds of config 4
# and config 2 over bench.py argument sets (SET: space-free, comma-separated args, "-" = none;
# e.g. "--adamw=plain", "--opt=pool_fuse=0" or "--lib=$PWD/ab_base.so").
#   usage: bash tools/gpu_r06d.sh TAG "PYTEST_K" ROUNDS "SET1" "SET2" ...
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; K=$2; N=$3; shift 3
mkdir -p gpurun_out
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -p no:cacheprovider -k "$K" > gpurun_out/$TAG.pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG.pytest.log | tail -2
  grep -E "^FAILED|^ERROR" gpurun_out/$TAG.pytest.log | head
  [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${CFGS:-c4 c2}; do
  if [ $cfg = c4 ]; then BA="--config 4 --mfma bf16 --steps 6 --warmup 2"; else BA="--steps 10 --warmup 3"; fi
  for r in $(seq 1 $N); do
    i=0
    for S in "$@"; do
      i=$((i+1))
      EXTRA=""; LIBV=""
      [ "$S" != "-" ] && EXTRA=$(echo "$S" | tr ',' ' ' | sed 's/--opt=/--opt /g; s/--adamw=/--adamw /g')
      # "--lib=PATH": run this set against another build of the library (UNET_HIP_LIB)
      case "$EXTRA" in *--lib=*) LIBV=$(echo "$EXTRA" | sed 's/.*--lib=\([^ ]*\).*/\1/'); EXTRA=$(echo "$EXTRA" | sed 's/--lib=[^ ]*//');; esac
      UNET_HIP_LIB=${LIBV:-$GRAFT_REPO_ROOT/thyroid-nodule-image-segmentation-unet-ddti_amd/lib/libunet_hip.so} \
      timeout -k 10 300 python bench.py --no-cpu-baseline --verbose $BA $EXTRA \
        > gpurun_out/$TAG.$cfg.r$r.s$i.json 2> gpurun_out/$TAG.$cfg.r$r.s$i.err
      rc=$?
      echo "$cfg round $r set $i [$S] rc=$rc: $(python -c "import json;d=json.load(open('gpurun_out/$TAG.$cfg.r$r.s$i.json'));print(d['value'],d['ms_per_step'])" 2>/dev/null)"
      [ $rc -ne 0 ] && { tail -n 20 gpurun_out/$TAG.$cfg.r$r.s$i.err; exit $rc; }
    done
  done
done
exit 0
