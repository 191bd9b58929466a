# MSD fused time-expansion conv (stts_conv1d_fwd_tx): its parity tests, the training suites it feeds, and the
# config-5 step with FUSE_TX off / on
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_layers.py tests/test_gpu_train_step.py tests/test_gpu_train_pred.py tests/test_gpu_msd.py -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tx.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_tx.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16,bf16x3 --no-fuse-tx --no-grad-check > gpurun_out/bench_tx_off.log 2>&1 || exit 3
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16,bf16x3,fp32 > gpurun_out/bench_tx_on.log 2>&1 || exit 3
tail -3 gpurun_out/bench_tx_off.log | cut -c1-600; tail -3 gpurun_out/bench_tx_on.log | cut -c1-900
