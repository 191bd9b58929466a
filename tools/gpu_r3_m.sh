# Round-3 batch: discriminator conv + leaky ReLU fused (stts_conv1d_fwd_act): training parity, step bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_layers.py tests/test_gpu_train_conv.py tests/test_gpu_train_step.py tests/test_gpu_mpd.py tests/test_gpu_msd.py -q -x -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_m.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_m.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_train_step.py --dtypes bf16 --steps 5 --warmup 2 > gpurun_out/bench_train_m.log 2>&1 || exit $?
cut -c1-200 gpurun_out/bench_train_m.log | grep config5
