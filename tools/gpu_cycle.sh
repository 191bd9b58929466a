# one build->measure cycle on the GPU box: parity tests, bench line, rocprofv3 kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/prof/bench_trace.log 2>&1 || exit $?
echo done
