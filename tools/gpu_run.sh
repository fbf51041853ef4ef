set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu2.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/gpu2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/bench2.json 2> gpurun_out/bench2.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench2.json; tail -30 gpurun_out/bench2.err
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof2 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof2.log 2>&1
echo "rocprof rc=$?"
ls -R $R/gpurun_out/prof2 | head
