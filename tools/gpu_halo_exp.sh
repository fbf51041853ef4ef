# GPU-box script: the halo x3 GEMM schedule experiments (tools/x3_halo_exp.hip), then one
# rocprofv3 PMC pass over the listed flag variants.
#   usage: bash tools/gpu_halo_exp.sh TAG "FLAGS" ["PMC FLAGS"] ["COUNTERS"]
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-hx}
FL=${2:-0,7,15,1,2,4,8,16,32,64,80}
PF=${3:-}
CN=${4:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE}
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3_halo_exp.hip -o /tmp/x3_halo_exp > gpurun_out/$TAG.build.log 2>&1 || { tail -20 gpurun_out/$TAG.build.log; exit 1; }
timeout -k 10 300 /tmp/x3_halo_exp 10 $FL > gpurun_out/$TAG.txt 2>&1
rc=$?
cat gpurun_out/$TAG.txt
[ $rc -ne 0 ] && exit $rc
[ -z "$PF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $CN --output-format csv -d $R/gpurun_out/$TAG.pmc -o run -- /tmp/x3_halo_exp 2 $PF > $R/gpurun_out/$TAG.pmc.log 2>&1
rc=$?
echo "pmc rc=$rc"; [ $rc -ne 0 ] && { tail -20 $R/gpurun_out/$TAG.pmc.log; exit $rc; }
python3 - $R/gpurun_out/$TAG.pmc <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "halo_exp" not in k and "row3_kernel" not in k: continue
    key = (k[:90], r.get("Grid_Size", ""))
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"]); n[(key, r["Counter_Name"])] += 1
for key, d in acc.items():
    print(key[0], "grid", key[1])
    print("   " + "  ".join(f"{c}={v / n[(key, c)]:.4g}" for c, v in sorted(d.items())))
PY
