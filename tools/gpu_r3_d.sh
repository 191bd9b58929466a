# Round-3 batch: plain-resconv / window-wgrad tests, conv A/B at config-5 shapes, train-step bench + profile.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_conv.py tests/test_gpu_train_step.py -q -x -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_train.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_train_conv.py --opt 15 > gpurun_out/ab_wgrad.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_train_conv.py --opt 16 > gpurun_out/ab_plainrc.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_train_step.py --dtypes bf16 --steps 5 --warmup 2 > gpurun_out/bench_train.log 2>&1 || exit $?
cut -c1-200 gpurun_out/bench_train.log | grep config5
rm -rf gpurun_out/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o train --output-format csv -- python3 tools/bench_train_step.py --dtypes bf16 --steps 3 --warmup 1 > gpurun_out/prof_train.log 2>&1 || exit $?
echo prof ok
