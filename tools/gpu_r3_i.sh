# Round-3 batch: latency fixes in the training step's small kernels (linear fwd / ds, bias column sums):
# training-layer + step parity, then the config-5 step bench (bf16).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_layers.py tests/test_gpu_train_conv.py tests/test_gpu_train_step.py -q -x -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_i.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_i.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_train_step.py --dtypes bf16 --steps 5 --warmup 2 > gpurun_out/bench_train_i.log 2>&1 || exit $?
cut -c1-400 gpurun_out/bench_train_i.log | grep config5
