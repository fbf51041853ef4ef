# GPU-box experiment script: optional tests, then bench A/B over environment settings
# (per-layer breakdown in the .err files), then the GEMM tile tuner.
# usage: bash tools/gpu_exp.sh TAG [tests] [tune] -- ENV_SETTING ...   ("-" = defaults)
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; shift
TESTS=0; TUNE=0
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  case $1 in tests) TESTS=1;; tune) TUNE=1;; esac; shift
done
[ $# -gt 0 ] && shift
if [ $TESTS = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/$TAG.pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/$TAG.pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for E in "$@"; do
  i=$((i+1))
  [ "$E" = "-" ] && E="UNET_AB_NONE=1"
  env $E timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verbose --no-cpu-baseline \
    > gpurun_out/$TAG.b$i.json 2> gpurun_out/$TAG.b$i.err
  rc=$?
  echo "bench $i [$E] rc=$rc: $(python -c "import json;d=json.load(open('gpurun_out/$TAG.b$i.json'));print(d['value'],d['ms_per_step'])" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -n 20 gpurun_out/$TAG.b$i.err; exit $rc; }
done
if [ $TUNE = 1 ]; then
  timeout -k 10 600 ./tools/gemm_tune 3 > gpurun_out/$TAG.tune.txt 2>&1
  rc=$?; echo "tune rc=$rc"; cat gpurun_out/$TAG.tune.txt
fi
