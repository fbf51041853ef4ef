# GPU-box script: bandwidth experiments on the x3 image pass (tools/x3_pass_exp.hip).
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-px}
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3_pass_exp.hip -o /tmp/x3_pass_exp > gpurun_out/$TAG.build.log 2>&1 || { tail -20 gpurun_out/$TAG.build.log; exit 1; }
timeout -k 10 300 /tmp/x3_pass_exp 20 > gpurun_out/$TAG.txt 2>&1
rc=$?
cat gpurun_out/$TAG.txt
exit $rc
