# HBM traffic of the dominant conv kernel (FETCH_SIZE / WRITE_SIZE in separate --pmc passes,
# kernel-trace only) over one bench step, reduced by tools/pmc_traffic.py into profiles/.
#   KERNEL=k_bigconv OUT=profiles/r01_traffic.json bash tools/gpu/gpu_traffic.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K=${KERNEL:-k_bigconv}
OUT=${OUT:-gpurun_out/traffic.json}
mkdir -p gpurun_out/traffic
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE -d gpurun_out/traffic/fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/traffic/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-include-regex "$K" --pmc WRITE_SIZE -d gpurun_out/traffic/write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/traffic/write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py gpurun_out/traffic "$K" "$OUT"
