# the reference's inference.py unit end to end (tokens -> waveform, B = 1, 10 s): tools/bench_duration.py and
# tools/e2e_breakdown.py, after the small-batch branch / decoder / graph suites
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_branches.py tests/test_gpu_decoder.py tests/test_gpu_graph.py tests/test_gpu_duration.py tests/test_gpu_edge.py -q -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_e2e.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_e2e.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/bench_duration.py --no-cpu-baseline > gpurun_out/bench_duration.log 2>&1 || exit $?
tail -1 gpurun_out/bench_duration.log | cut -c1-400
timeout -k 10 300 python -u tools/e2e_breakdown.py > gpurun_out/e2e_breakdown.log 2>&1 || exit $?
tail -15 gpurun_out/e2e_breakdown.log
