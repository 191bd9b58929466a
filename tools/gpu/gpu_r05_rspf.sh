# Round 5: ressplit epilogue-row prefetch (STTS_OPT_EXP 16384) vs off, bf16x3, + the split parity tests with it on
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
STTS_OPTS=13=16384 timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -m gpu -k "ressplit or big64 or config3 or golden" -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rspf.log 2>&1 || { tail -20 gpurun_out/pytest_rspf.log; exit 3; }
tail -2 gpurun_out/pytest_rspf.log
timeout -k 10 400 python -u tools/ab_engine.py 13 0 16384 --rounds 2 --dtype bf16x3 > gpurun_out/ab_rspf.log 2>&1 || { tail -20 gpurun_out/ab_rspf.log; exit 3; }
grep -E "^opt|ressplit'" gpurun_out/ab_rspf.log
