# Round 5: STTS_OPT_BIGCONV (7) 2 (default: v1 for C = 128 k3) vs 3 (bigconv2 4-wave blocks everywhere) vs 4 (8-wave everywhere), bf16
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_engine.py 7 2 3 4 --rounds 3 > gpurun_out/ab_bigmode.log 2>&1 || { tail -20 gpurun_out/ab_bigmode.log; exit 3; }
grep -E "^opt|k_bigconv', 128" gpurun_out/ab_bigmode.log | head -40
