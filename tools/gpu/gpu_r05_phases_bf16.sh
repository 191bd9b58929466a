# Round 5: bigconv2 phase attribution in bf16 (STTS_OPT_DEBUG skip bits, timing only; outputs wrong while set):
# 128 epilogue stores, 4 whole epilogue, 1 window transform, 32 group barrier, 8 weight DMAs, 16 window DMAs, 61 all but MFMA
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_engine.py 4 0 128 4 1 32 8 16 61 --rounds 2 > gpurun_out/phases_bf16.log 2>&1 || { tail -20 gpurun_out/phases_bf16.log; exit 3; }
grep -E "k_bigconv|^opt" gpurun_out/phases_bf16.log | head -60
