# STTS_OPT_BRANCHES batch threshold: bench lines at B = 8, 16, 32 with the concurrent branches off / forced on
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
A="--steps 10 --warmup 3 --no-cpu-baseline --no-parity-mode --no-accuracy-mode --no-e2e --no-profile"
for b in 8 16 32; do
  STTS_OPTS=23=0 timeout -k 10 300 python -u bench.py --batch $b $A > gpurun_out/bench_sw_b${b}_off.log 2>&1 || exit 3
  STTS_OPTS=23=64 timeout -k 10 300 python -u bench.py --batch $b $A > gpurun_out/bench_sw_b${b}_on.log 2>&1 || exit 3
  echo "B=$b off: $(tail -1 gpurun_out/bench_sw_b${b}_off.log | cut -c1-190)"
  echo "B=$b on:  $(tail -1 gpurun_out/bench_sw_b${b}_on.log | cut -c1-190)"
done
