# the noise branches alone on a side stream at B = 16 / 32 (STTS_OPT_NBRANCH) vs none, bench lines in one box
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode --no-accuracy-mode --no-e2e --no-profile"
for b in 16 32; do
  for o in 0 64 0 64; do
    STTS_OPTS=24=$o timeout -k 10 300 python -u bench.py --batch $b $A > gpurun_out/bench_nb_b${b}_$o.log 2>&1 || exit 3
    echo "B=$b nbranch=$o: $(tail -1 gpurun_out/bench_nb_b${b}_$o.log | cut -c100-190)"
  done
done
