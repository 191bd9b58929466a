# Full measurement cycle on the GPU box: parity tests, default bench line (with the CPU baseline),
# per-launch layer table, rocprofv3 kernel-trace stats of the same bench command, and the HBM
# traffic passes of the dominant kernel.  Every GPU step has its own limit; the first failure ends it.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-600
timeout -k 10 300 python tools/layer_profile.py > gpurun_out/layers.txt 2>&1 || exit 1
tail -1 gpurun_out/layers.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof/bench_trace.log 2>&1 || { tail -20 gpurun_out/prof/bench_trace.log; exit 1; }
tail -1 gpurun_out/prof/bench_trace.log | cut -c1-300
KERNEL=${KERNEL:-k_bigconv} OUT=gpurun_out/traffic.json bash tools/gpu_traffic.sh || exit 1
echo done
