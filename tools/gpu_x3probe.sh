# GPU-box script: split-bf16 fp32 GEMM probe (tools/x3_probe.hip) vs the f32 pipelined kernel.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-x3}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3_probe.hip -o /tmp/x3_probe 2> gpurun_out/$TAG.build.log || { tail -20 gpurun_out/$TAG.build.log; exit 1; }
timeout -k 10 240 /tmp/x3_probe 5 > gpurun_out/$TAG.probe.txt 2>&1
rc=$?
cat gpurun_out/$TAG.probe.txt
exit $rc
