# round-4 A/B cycle: the C32 weight gradient (training) and the bigconv2 offset halves (STTS_OPT_BIGCONV 5)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_conv.py tests/test_gpu_train_step.py "tests/test_gpu_conv.py::test_bigconv_v2_matches_v1" "tests/test_gpu_conv.py::test_bigconv_8wave_many_tiles_per_workgroup" -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ab2.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/ab_engine.py 7 2 5 --rounds 3 > gpurun_out/ab_ofs.log 2>&1 || exit 3
grep "^opt" gpurun_out/ab_ofs.log
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16 --opt 13=4096 --no-grad-check > gpurun_out/bench_train_c32a.log 2>&1 || exit 3
timeout -k 10 400 python -u tools/bench_train_step.py --steps 6 --warmup 2 --dtypes bf16 --no-grad-check > gpurun_out/bench_train_c32b.log 2>&1 || exit 3
tail -1 gpurun_out/bench_train_c32a.log | cut -c1-300; tail -1 gpurun_out/bench_train_c32b.log | cut -c1-300
