# Round-2 closing cycle on the MI355X: the -m gpu suite, the dominant kernel's HBM traffic (separate
# FETCH_SIZE / WRITE_SIZE passes, copied into profiles/ on the box so the bench line carries it), the
# default bench line, and the same bench under rocprofv3 --kernel-trace --stats.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
KERNEL=k_bigconv OUT=gpurun_out/traffic.json bash tools/gpu_traffic.sh > gpurun_out/traffic.log 2>&1 || exit $?
cp gpurun_out/traffic.json profiles/r02_traffic.json
echo "traffic ok"
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
rm -rf gpurun_out/prof_bench
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
echo "profiled bench ok"
