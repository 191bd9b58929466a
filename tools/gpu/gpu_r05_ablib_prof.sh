# Round 5: per-kernel rocprofv3 stats of bench.py (decode only) with another build (A) and this tree's (B)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
other=$1; shift
for v in A B; do
  if [ $v = A ]; then export STTS_LIB=$PWD/$other; else unset STTS_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abprof_$v -o run -- python3 bench.py --no-cpu-baseline \
    --no-profile --no-parity-mode --no-accuracy-mode --no-e2e "$@" > gpurun_out/abprof_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/abprof_$v -name "*kernel_stats.csv" | head -1)
  cp $f gpurun_out/abprof_${v}_kernel_stats.csv
  head -14 $f | cut -d, -f1-4
done
