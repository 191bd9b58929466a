# Round-6 closing cycle on the MI355X, in two calls (each under gpurun's time limit):
#   PART=a: the default bench line, the same bench under rocprofv3 --kernel-trace --stats
#   PART=b: SQ counter passes of the two headline engine families, and B = 1 with / without
#           the concurrent resblock branches (the config-5 step: tools/gpu/gpu_r06_train_eg.sh)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${PART:-a}" = "a" ]; then
  # (the -m gpu suite and smoke: tools/gpu/gpu_r06_suite.sh, its own call)
  timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
  tail -1 gpurun_out/bench.log | cut -c1-300
  rm -rf gpurun_out/prof_bench
  # (the whole process with the noise-branch overlap off, STTS_OPT_NBRANCH = 24 = 0, as the bench's own profiled pass:
  # rocprofv3's per-kernel averages then price each launch alone and agree with the line's avg_launch_us)
  STTS_OPTS=24=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
  echo "profiled bench ok"
else
  export BENCH_ARGS="--no-parity-mode --no-accuracy-mode --no-e2e"
  export STTS_OPTS=24=0  # counters of each launch alone
  for fam in k_bigconv k_resconv; do
    rm -rf gpurun_out/pmc
    KREGEX=$fam timeout -k 10 600 bash tools/gpu/gpu_pmc.sh > gpurun_out/pmc_r06_$fam.log 2>&1 || exit $?
    python3 tools/analyze_pmc.py gpurun_out/pmc > gpurun_out/pmc_${fam}_r06.txt 2>&1 || exit $?
    rm -rf gpurun_out/pmc_$fam && mv gpurun_out/pmc gpurun_out/pmc_$fam
  done
  echo pmc ok
  unset STTS_OPTS
  # B = 1 (the reference's inference.py unit): concurrent resblock branches (default) vs the running sum
  B1="--batch 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-mode --no-accuracy-mode --no-e2e --no-profile"
  STTS_OPTS=23=0,24=0 timeout -k 10 300 python -u bench.py $B1 > gpurun_out/bench_b1_nobranch.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py $B1 > gpurun_out/bench_b1_branch.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_b1_nobranch.log | cut -c1-250; tail -1 gpurun_out/bench_b1_branch.log | cut -c1-250
fi
