# Round-4 closing cycle on the MI355X: the -m gpu suite, smoke, the dominant kernel's HBM traffic (separate
# FETCH_SIZE / WRITE_SIZE passes reduced with the round-3 counter calibration), the default bench line, the same
# bench under rocprofv3 --kernel-trace --stats, SQ counter passes of the two headline engine families, and the
# config-5 training step (bf16 with the gradient check against fp32, and fp32).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
  tail -3 gpurun_out/pytest_gpu.log
  [ $rc -le 1 ] || exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
  tail -1 gpurun_out/smoke.log
fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
rm -rf gpurun_out/prof_bench
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
echo "profiled bench ok"
if [ -z "$SKIP_PMC" ]; then
  KERNEL=k_bigconv OUT=gpurun_out/traffic.json bash tools/gpu_traffic.sh > gpurun_out/traffic.log 2>&1 || exit $?
  export BENCH_ARGS="--no-parity-mode --no-accuracy-mode --no-e2e"
  for fam in k_bigconv k_resconv; do
    rm -rf gpurun_out/pmc
    KREGEX=$fam timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/pmc_r04_$fam.log 2>&1 || exit $?
    python3 tools/analyze_pmc.py gpurun_out/pmc > gpurun_out/pmc_${fam}_r04.txt 2>&1 || exit $?
    rm -rf gpurun_out/pmc_$fam && mv gpurun_out/pmc gpurun_out/pmc_$fam
  done
  echo pmc ok
fi
timeout -k 10 600 python -u tools/bench_train_step.py --steps 8 --warmup 2 --dtypes bf16,bf16x3,fp32 > gpurun_out/bench_train_r04.log 2>&1 || exit $?
tail -2 gpurun_out/bench_train_r04.log | cut -c1-400
