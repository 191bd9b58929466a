# Round 5: bigconv2 phase attribution by STTS_OPT_DEBUG skip bits (timing only; outputs wrong while set):
# 128 epilogue stores, 4 whole epilogue, 1 window transform, 256 statistics, 32 group barrier, 8 weight DMAs, 16 window DMAs
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_engine.py 4 0 128 4 1 256 32 8 16 --rounds 2 > gpurun_out/phases_bf16.log 2>&1 || { tail -20 gpurun_out/phases_bf16.log; exit 3; }
grep -E "k_bigconv|^opt" gpurun_out/phases_bf16.log | head -60
timeout -k 10 300 python -u tools/ab_engine.py 4 0 128 4 1 32 8 --rounds 1 --dtype bf16x3 > gpurun_out/phases_split.log 2>&1 || { tail -20 gpurun_out/phases_split.log; exit 3; }
grep -E "k_bigconv|^opt" gpurun_out/phases_split.log | head -40
