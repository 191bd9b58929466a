# Round 5: C = 64 resblock convs on bigconv2 (NF = 4): parity tests, then in-process A/Bs (bf16x3: BIG64 1 vs 0; bf16: 2 vs 0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_decoder.py -m gpu -k "big64 or ressplit or bigsplit or deterministic" -q -rfE -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_big64.log 2>&1 || { grep -E "passed|failed|Error|^E " gpurun_out/pytest_big64.log | tail -30; exit 3; }
grep -E "passed|failed|big64" gpurun_out/pytest_big64.log | tail -12
timeout -k 10 400 python -u tools/ab_engine.py 27 1 0 --rounds 2 --dtype bf16x3 > gpurun_out/ab_big64_split.log 2>&1 || { tail -20 gpurun_out/ab_big64_split.log; exit 3; }
grep -E "^opt|k_bigconv2\[SP\]', 64|k_ressplit', 64" gpurun_out/ab_big64_split.log | head -40
timeout -k 10 400 python -u tools/ab_engine.py 27 2 0 --rounds 3 > gpurun_out/ab_big64_bf16.log 2>&1 || { tail -20 gpurun_out/ab_big64_bf16.log; exit 3; }
grep -E "^opt|k_bigconv', 64|k_resconv', 64" gpurun_out/ab_big64_bf16.log | head -40
