# rocprofv3 kernel trace + HBM counters of the default bench workload (1 timed step).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/bench_trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/bench_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/bench_write.log 2>&1 || exit $?
find gpurun_out/prof -name "*.csv" | head -20
