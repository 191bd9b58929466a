# Round-3 batch: training-path tests (new all-taps bf16 weight-gradient kernel), the config-5 step bench,
# the headline bench line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_conv.py tests/test_gpu_train_layers.py tests/test_gpu_train_step.py -q -x -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_train.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_train_step.py --dtypes bf16,fp32 --steps 5 --warmup 2 > gpurun_out/bench_train.log 2>&1 || exit $?
cut -c1-260 gpurun_out/bench_train.log | grep config5
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
