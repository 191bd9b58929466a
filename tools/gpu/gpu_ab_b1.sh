cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_engine.py 5 16 4 1 32 --batch 1 --rounds 3 > gpurun_out/ab_b1_slots.log 2>&1 || exit 3
grep "^opt" gpurun_out/ab_b1_slots.log
timeout -k 10 300 python -u tools/ab_engine.py 7 2 3 --batch 1 --rounds 3 > gpurun_out/ab_b1_bigconv.log 2>&1 || exit 3
grep "^opt" gpurun_out/ab_b1_bigconv.log
timeout -k 10 300 python -u tools/ab_engine.py 2 0 512 1024 --batch 1 --rounds 3 > gpurun_out/ab_b1_grid.log 2>&1 || exit 3
grep "^opt" gpurun_out/ab_b1_grid.log
