# small-batch decoder concurrency (STTS_OPT_BRANCHES: resblock branches + noise branches on side streams): the
# decoder / graph / branch suites, then B = 1 and B = 4 bench lines with the option off and on
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_branches.py tests/test_gpu_decoder.py tests/test_gpu_graph.py tests/test_gpu_split.py -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_br.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_br.log; [ $rc -le 1 ] || exit $rc
A="--steps 20 --warmup 5 --no-cpu-baseline --no-parity-mode --no-accuracy-mode --no-e2e --no-profile"
for b in 1 4; do
  STTS_OPTS=23=0 timeout -k 10 300 python -u bench.py --batch $b $A > gpurun_out/bench_br_b${b}_off.log 2>&1 || exit 3
  timeout -k 10 300 python -u bench.py --batch $b $A > gpurun_out/bench_br_b${b}_on.log 2>&1 || exit 3
  tail -1 gpurun_out/bench_br_b${b}_off.log | cut -c1-200; tail -1 gpurun_out/bench_br_b${b}_on.log | cut -c1-200
done
