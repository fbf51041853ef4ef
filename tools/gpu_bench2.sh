# GPU-box script: the two benches only (config 2 without CPU baseline, config 4 bf16).
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-b2}
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verbose --no-cpu-baseline > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?
echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/$TAG.bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'])"; grep -E "^  conv|^  convT" gpurun_out/$TAG.bench.err | head -6
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config 4 --mfma bf16 --steps 4 --warmup 2 --verbose --no-cpu-baseline > gpurun_out/$TAG.c4bf16.json 2> gpurun_out/$TAG.c4bf16.err
rc=$?
echo "bench c4 rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/$TAG.c4bf16.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'])"; grep -v amdgpu.ids gpurun_out/$TAG.c4bf16.err | head -16
exit $rc
