# Round 5: the accuracy mode's C = 32 convs on bigconv2 (NF = 2, 4-wave blocks; STTS_OPT_BIG64 bit 8) vs ressplit
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_engine.py 27 5 13 --rounds 2 --dtype bf16x3 > gpurun_out/ab_big32.log 2>&1 || { tail -20 gpurun_out/ab_big32.log; exit 3; }
grep -E "^opt|SP\]', 32|ressplit', 32" gpurun_out/ab_big32.log
