# Round-3: MSD engine fold (tests + A/B).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_train_step.py tests/test_gpu_train_conv.py -q -x -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_msd.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_msd.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_msd_fold.py > gpurun_out/ab_msd_fold.log 2>&1 || exit $?
tail -1 gpurun_out/ab_msd_fold.log
timeout -k 10 300 python -u tools/bench_train_step.py --dtypes bf16 --steps 5 --warmup 2 > gpurun_out/bench_train.log 2>&1 || exit $?
cut -c1-200 gpurun_out/bench_train.log | grep config5
