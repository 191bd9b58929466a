# training-path GPU cycle: parity suites, then the config-5 step with an engine option A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
STTS_OPTS=${TEST_OPTS:-20=1} timeout -k 10 900 python -u -m pytest ${TRAIN_TESTS:-tests/test_gpu_train_conv.py tests/test_gpu_train_layers.py tests/test_gpu_train_step.py} -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_train.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16 --opt ${AB_OPT:-20}=${AB_A:-0} > gpurun_out/bench_train_a.log 2>&1 || exit 3
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16,bf16x3,fp32 --opt ${AB_OPT:-20}=${AB_B:-1} > gpurun_out/bench_train_b.log 2>&1 || exit 3
tail -2 gpurun_out/bench_train_a.log | cut -c1-700; tail -2 gpurun_out/bench_train_b.log | cut -c1-900
