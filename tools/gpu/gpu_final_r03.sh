# Round-3 closing cycle on the MI355X: the -m gpu suite, smoke, the dominant kernel's HBM traffic
# (separate FETCH_SIZE / WRITE_SIZE passes, reduced with the round-3 counter calibration), the default
# bench line, the same bench under rocprofv3 --kernel-trace --stats, and the other configs.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
KERNEL=k_bigconv OUT=gpurun_out/traffic.json bash tools/gpu/gpu_traffic.sh > gpurun_out/traffic.log 2>&1 || exit $?
python3 tools/traffic_calibrated.py gpurun_out/traffic profiles/r03_calib_c256.json profiles/r03_calib_c128.json profiles/r03_traffic.json > profiles/r03_traffic_calibrated.txt 2>&1 || exit $?
tail -1 profiles/r03_traffic_calibrated.txt
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
rm -rf gpurun_out/prof_bench
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
echo "profiled bench ok"
