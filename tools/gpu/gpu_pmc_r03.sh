# Round-3 PMC passes (SQ counters only; HBM bytes are in profiles/r03_traffic*.json) of the two headline
# engine families over one bench step: k_bigconv (mfmabusy, waits) and k_resconv.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export BENCH_ARGS="--no-parity-mode --no-e2e"
mkdir -p gpurun_out
for fam in k_bigconv k_resconv; do
  rm -rf gpurun_out/pmc
  KREGEX=$fam timeout -k 10 900 bash tools/gpu/gpu_pmc.sh > gpurun_out/pmc_r03_$fam.log 2>&1 || exit $?
  python3 tools/analyze_pmc.py gpurun_out/pmc > gpurun_out/pmc_${fam}_r03.txt 2>&1 || exit $?
  rm -rf gpurun_out/pmc_$fam && mv gpurun_out/pmc gpurun_out/pmc_$fam
done
echo pmc ok
