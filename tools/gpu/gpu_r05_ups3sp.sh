# Round 5: the accuracy mode's ups[3] (N = 64) on bigconv2 SP (NCB = 1, NF = 2): split parity tests + A/B UPS 1 vs 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -m gpu -q -rfE -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ups3sp.log 2>&1 || { grep -E "passed|failed|^E |Error" gpurun_out/pytest_ups3sp.log | tail -20; exit 3; }
grep -E "passed|bigsplit A/B|10 s|golden" gpurun_out/pytest_ups3sp.log | tail -12
timeout -k 10 400 python -u tools/ab_engine.py 14 1 2 --rounds 2 --dtype bf16x3 > gpurun_out/ab_ups3sp.log 2>&1 || { tail -20 gpurun_out/ab_ups3sp.log; exit 3; }
grep -E "^opt|, (192|64), 2, " gpurun_out/ab_ups3sp.log
