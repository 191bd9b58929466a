# Round 5: build-against-build A/B on one box (arg 1: the other library; arg 2: dtype; rest: bench args).
# Runs bench.py (decode only) alternately with the other build (A) and this tree's (B), 3 rounds.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
other=$1; dt=$2; shift 2
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=$PWD/$other; else lib=; fi
    STTS_LIB=$lib timeout -k 10 300 python -u bench.py --dtype $dt --no-cpu-baseline --no-profile --no-parity-mode \
      --no-accuracy-mode --no-e2e "$@" > gpurun_out/ablib_$v$r.json 2> gpurun_out/ablib_$v$r.err || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/ablib_$v$r.json').read().strip().splitlines()[-1]); print('$v$r', '$dt', d['value']/1e6, d['ms_per_step'], d.get('ms_per_step_median'))"
  done
done
