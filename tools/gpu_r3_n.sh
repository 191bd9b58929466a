# Round-3 batch: stride-2 narrow-N igemm tile (BM 128 x BN 32): conv / training / discriminator parity, step bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train_conv.py tests/test_gpu_train_step.py tests/test_gpu_mpd.py tests/test_gpu_msd.py tests/test_gpu_decoder.py -q -x -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_n.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_n.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_train_step.py --dtypes bf16 --steps 5 --warmup 2 > gpurun_out/bench_train_n.log 2>&1 || exit $?
cut -c1-200 gpurun_out/bench_train_n.log | grep config5
