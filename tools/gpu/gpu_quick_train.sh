# training-step check after a host-side change: the step / predictor / graph suites, then the config-5 bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${QT_TESTS:-tests/test_gpu_train_step.py tests/test_gpu_train_pred.py tests/test_gpu_graph.py} -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_qt.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_qt.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes ${QT_DT:-bf16,bf16x3,fp32} ${QT_ARGS:-} > gpurun_out/bench_qt.log 2>&1 || exit 3
grep -h ms_per_step gpurun_out/bench_qt.log | cut -c1-230
