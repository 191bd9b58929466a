# Round-2 GPU cycle: the -m gpu suite, the default bench line, and the duration bench under
# rocprofv3 with the B = 1 (cooperative BiLSTM) leg included.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-600
mkdir -p gpurun_out/prof_dur
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dur -o dur --output-format csv -- python3 tools/bench_duration.py --no-cpu-baseline --steps 5 > gpurun_out/prof_dur.log 2>&1
echo "profiled duration bench rc=$?"
