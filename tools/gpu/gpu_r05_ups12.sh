# Round 5: ups[2] on 12-wave bigconv2 blocks (default; STTS_OPT_EXP bit 32 = the 4-wave blocks) and the accuracy mode's
# ups[3] with both phases per tile (bit 64): layout parity tests, the ups / split suites, then in-process A/Bs
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_split.py tests/test_gpu_decoder.py -q -x -rA -k "ups or split or decoder" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ups12_pytest.log 2>&1 || { tail -30 gpurun_out/ups12_pytest.log; exit 3; }
grep -E "passed|failed|split ups layouts" gpurun_out/ups12_pytest.log | tail -8
bash tools/gpu/gpu_r05_ab.sh 13 32 0 64 || exit 3
grep -E "192|, 64, 2,|^opt" gpurun_out/ab_bf16.log gpurun_out/ab_split.log
