# Round 6: the marginal cost of weight LDS-DMA pieces in the v3 engine (STTS_OPT_EXP bit 131072 issues every piece
# twice), and v3 vs bigconv2 once more on the same box
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_engine.py 13 0 131072 --rounds 3 --set 28=7 > gpurun_out/r06_ab_dma2x.txt 2>&1 || exit $?
grep "k_bigconv', \(128\|256\|1024\|2560\)\|^opt" gpurun_out/r06_ab_dma2x.txt | head -40
