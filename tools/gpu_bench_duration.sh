cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_dur
timeout -k 10 300 python tools/bench_duration.py > gpurun_out/bench_dur.log 2>&1 || exit $?
tail -1 gpurun_out/bench_dur.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dur -o dur --output-format csv -- python3 tools/bench_duration.py --no-cpu-baseline --no-e2e --steps 5 > gpurun_out/prof_dur.log 2>&1 || exit $?
find gpurun_out/prof_dur -name '*stats*'
