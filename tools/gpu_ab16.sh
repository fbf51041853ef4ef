# GPU-box script: config-4 bf16 bench under several environment settings (A/B), one line each.
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-ab}
shift
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python bench.py --config 4 --mfma bf16 --steps 4 --warmup 2 --verbose --no-cpu-baseline > gpurun_out/$TAG.$i.json 2> gpurun_out/$TAG.$i.err
  rc=$?
  echo "[$E] rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/$TAG.$i.json'));print(d['value'], d['ms_per_step'])")"
  grep -E "conv_wgrad  |conv_dgrad  |conv_fwd  |convT" gpurun_out/$TAG.$i.err | head -6
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/$TAG.$i.err; exit $rc; fi
done
