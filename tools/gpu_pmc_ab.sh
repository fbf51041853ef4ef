# GPU-box script: one rocprofv3 PMC pass (FETCH_SIZE + WRITE_SIZE need two passes: TCC slots)
# per option arm of a bench workload, summarised per kernel (tools/pmc_summary.py).
# usage: bash tools/gpu_pmc_ab.sh TAG "BENCH ARGS" KERNEL "opt=v ..." ...   ("-" = defaults)
set -u
R=$GRAFT_REPO_ROOT
TAG=$1; BARGS=$2; KERN=$3; shift 3
cd /tmp && export TMPDIR=/tmp
i=0
for A in "$@"; do
  i=$((i+1))
  OPTS=""
  if [ "$A" != "-" ]; then for kv in $A; do OPTS="$OPTS --opt $kv"; done; fi
  j=0
  for CN in "FETCH_SIZE" "WRITE_SIZE"; do
    j=$((j+1))
    timeout -s KILL 240 rocprofv3 --pmc $CN --output-format csv -d $R/gpurun_out/$TAG.$i.pmc$j -o run -- python3 $R/bench.py $BARGS --no-cpu-baseline $OPTS > $R/gpurun_out/$TAG.$i.pmc$j.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "[$A] pmc $CN rc=$rc"; tail -5 $R/gpurun_out/$TAG.$i.pmc$j.log; exit $rc; fi
  done
  (cd $R && python3 tools/pmc_summary.py gpurun_out/$TAG.$i.json gpurun_out/$TAG.$i.pmc1 gpurun_out/$TAG.$i.pmc2 > /dev/null && \
   python3 -c "
import json; d=json.load(open('gpurun_out/$TAG.$i.json'))['kernels']
for k in sorted(d, key=lambda k: -d[k].get('hbm_bytes_per_launch', 0) * d[k].get('dispatches', 0))[:6]:
    v=d[k]; print('[$A]', k, 'GB/launch %.3f' % (v.get('hbm_bytes_per_launch', 0)/1e9), 'ms %.3f' % (v.get('avg_duration_ns_profiled', 0)/1e6), 'n', v.get('dispatches'))
")
done
