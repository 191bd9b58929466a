# MSD time expansion inside the convs (stts_conv1d_fwd_tx / _bwd_tx / _wgrad_tx) and fp32 output frames of the
# bf16 general-engine convs (STTS_OPT_YF32): the training parity suites, then the config-5 step with both off,
# YF32 alone, and both on (the defaults)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_conv.py tests/test_gpu_train_layers.py tests/test_gpu_train_step.py tests/test_gpu_train_pred.py tests/test_gpu_msd.py -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tx.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_tx.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16 --no-fuse-tx --opt 21=0 --no-grad-check > gpurun_out/bench_tx_base.log 2>&1 || exit 3
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16 --no-fuse-tx --no-grad-check > gpurun_out/bench_tx_yf.log 2>&1 || exit 3
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16,bf16x3,fp32 > gpurun_out/bench_tx_on.log 2>&1 || exit 3
for f in base yf on; do grep -h ms_per_step_median gpurun_out/bench_tx_$f.log | cut -c1-150; done
