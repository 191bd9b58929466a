# Round 5: ups[2] (N = 192) on bigconv2 (NCB = 2, NF = 4, 4-wave blocks): parity tests, then A/B STTS_OPT_UPS 1 vs 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_split.py tests/test_gpu_decoder.py -m gpu -k "ups or bigsplit or golden or deterministic or matches_reference" -q -rfE -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ups2.log 2>&1 || { grep -E "passed|failed|^E |Error" gpurun_out/pytest_ups2.log | tail -20; exit 3; }
tail -2 gpurun_out/pytest_ups2.log
timeout -k 10 400 python -u tools/ab_engine.py 14 1 2 --rounds 3 > gpurun_out/ab_ups2.log 2>&1 || { tail -20 gpurun_out/ab_ups2.log; exit 3; }
grep -E "^opt|, 192, " gpurun_out/ab_ups2.log
timeout -k 10 400 python -u tools/ab_engine.py 14 1 2 --rounds 2 --dtype bf16x3 > gpurun_out/ab_ups2_split.log 2>&1 || { tail -20 gpurun_out/ab_ups2_split.log; exit 3; }
grep -E "^opt|, 192, " gpurun_out/ab_ups2_split.log
