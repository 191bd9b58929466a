# sub-discriminators on their own HIP streams (discriminators.CONCURRENT): the training parity suites, then the
# config-5 step serial vs concurrent
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_train_pred.py tests/test_gpu_train_layers.py tests/test_gpu_msd.py tests/test_gpu_mpd.py -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_conc.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_conc.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16 --serial-discs --no-grad-check > gpurun_out/bench_conc_off.log 2>&1 || exit 3
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16,bf16x3,fp32 > gpurun_out/bench_conc_on.log 2>&1 || exit 3
for f in off on; do grep -h ms_per_step_median gpurun_out/bench_conc_$f.log | cut -c1-150; done
