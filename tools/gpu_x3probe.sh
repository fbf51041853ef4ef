# GPU-box script: split-bf16 fp32 GEMM probe (tools/x3_probe.hip) vs the f32 kernels.
#   usage: bash tools/gpu_x3probe.sh TAG [WHAT: 1 row GEMMs, 2 weight gradients, 3 both]
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-x3}
WHAT=${2:-3}
L=thyroid-nodule-image-segmentation-unet-ddti_amd/lib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3_probe.hip -o /tmp/x3_probe -L $L -lunet_hip 2> gpurun_out/$TAG.build.log || { tail -20 gpurun_out/$TAG.build.log; exit 1; }
LD_LIBRARY_PATH=$L:${LD_LIBRARY_PATH:-} timeout -k 10 300 /tmp/x3_probe 5 $WHAT > gpurun_out/$TAG.probe.txt 2>&1
rc=$?
cat gpurun_out/$TAG.probe.txt
exit $rc
