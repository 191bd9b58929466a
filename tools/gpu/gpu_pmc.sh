# SQ / TCC counters for the conv kernels of one bench step (separate passes, kernel-trace only)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS}"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-include-regex "${KREGEX:-conv1d_igemm}" --pmc "$@" -d gpurun_out/pmc/$name -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -le 1 ] || exit $rc
}
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run c SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA
run d FETCH_SIZE
run e WRITE_SIZE
find gpurun_out/pmc -name "*counter_collection.csv" | head
