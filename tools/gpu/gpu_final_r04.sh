# Round-4 closing cycle on the MI355X, in two calls (each under gpurun's time limit):
#   PART=a: the -m gpu suite, smoke, the default bench line, the same bench under rocprofv3 --kernel-trace --stats
#   PART=b: the dominant kernel's HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes, reduced with the round-3
#           counter calibration), SQ counter passes of the two headline engine families, and the config-5
#           training step (bf16 with the gradient check against fp32, bf16x3, fp32)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${PART:-a}" = "a" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
  tail -3 gpurun_out/pytest_gpu.log
  [ $rc -le 1 ] || exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
  tail -1 gpurun_out/smoke.log
  timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
  tail -1 gpurun_out/bench.log | cut -c1-300
  rm -rf gpurun_out/prof_bench
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
  echo "profiled bench ok"
else
  export BENCH_ARGS="--no-parity-mode --no-accuracy-mode --no-e2e"
  KERNEL=k_bigconv OUT=gpurun_out/traffic.json bash tools/gpu/gpu_traffic.sh > gpurun_out/traffic.log 2>&1 || exit $?
  for fam in k_bigconv k_resconv; do
    rm -rf gpurun_out/pmc
    KREGEX=$fam timeout -k 10 600 bash tools/gpu/gpu_pmc.sh > gpurun_out/pmc_r04_$fam.log 2>&1 || exit $?
    python3 tools/analyze_pmc.py gpurun_out/pmc > gpurun_out/pmc_${fam}_r04.txt 2>&1 || exit $?
    rm -rf gpurun_out/pmc_$fam && mv gpurun_out/pmc gpurun_out/pmc_$fam
  done
  echo pmc ok
  timeout -k 10 500 python -u tools/bench_train_step.py --steps 8 --warmup 2 --dtypes bf16,bf16x3,fp32 > gpurun_out/bench_train_r04.log 2>&1 || exit $?
  tail -3 gpurun_out/bench_train_r04.log | cut -c1-300
  timeout -k 10 300 python -u tools/train_conv_shapes.py --dtype bf16 --top 40 > gpurun_out/train_conv_shapes_r04.txt 2>&1 || exit $?
  head -3 gpurun_out/train_conv_shapes_r04.txt
  # B = 1 (the reference's inference.py unit): concurrent resblock branches (default) vs the running sum
  B1="--batch 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-mode --no-accuracy-mode --no-e2e --no-profile"
  STTS_OPTS=23=0 timeout -k 10 300 python -u bench.py $B1 > gpurun_out/bench_b1_nobranch.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py $B1 > gpurun_out/bench_b1_branch.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_b1_nobranch.log | cut -c1-250; tail -1 gpurun_out/bench_b1_branch.log | cut -c1-250
fi
