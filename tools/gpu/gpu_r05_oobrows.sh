# Round 5: price the window DMA's all-zero padding rows (STTS_OPT_DEBUG 512: not issued; timing only) in bf16
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_engine.py 4 0 512 --rounds 3 > gpurun_out/ab_oobrows.log 2>&1 || { tail -20 gpurun_out/ab_oobrows.log; exit 3; }
grep -E "^opt|k_bigconv'" gpurun_out/ab_oobrows.log
