# Round 6: C = 64 residual / running-sum launches (K >= 7) on the ping-pong kernel (STTS_OPT_RCPP 1, default) vs the
# lock-step kernel with the interleaved epilogue (3), in-process, 5 rounds
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_engine.py 18 1 3 --rounds 5 > gpurun_out/r06_ab_rcpp3.txt 2>&1 || exit $?
grep "^opt\|k_resconv', 64, \(7\|11\), 1, [13]" gpurun_out/r06_ab_rcpp3.txt
