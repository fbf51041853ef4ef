# A/B of environment settings on the same box: alternates bench runs.
# usage: bash tools/ab.sh TAG "ENV_A" "ENV_B" [rounds]   (ENV_x like "UNET_TILE_N128=4" or "-")
set -u
cd $GRAFT_REPO_ROOT
TAG=$1; A=$2; B=$3; N=${4:-2}
for r in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    if [ "$E" = "-" ]; then E="UNET_AB_NONE=1"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/$TAG.$v$r.json 2>/dev/null || exit $?
    python -c "import json; d=json.load(open('gpurun_out/$TAG.$v$r.json')); print('$v$r', '$E', d['value'], d['ms_per_step'])"
  done
done
