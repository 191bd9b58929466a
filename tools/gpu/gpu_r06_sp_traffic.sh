# Round 6: HBM traffic of the accuracy mode's dominant family (k_bigconv2[SP], bf16x3, B = 32 x 10 s)
# from separate FETCH_SIZE / WRITE_SIZE passes over one bench step, reduced by tools/pmc_traffic.py (reads 2 x FETCH)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sptraffic && export TMPDIR=/tmp
ARGS="--dtype bf16x3 --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-parity-mode --no-accuracy-mode --no-e2e"
timeout -s KILL 300 rocprofv3 --kernel-include-regex k_bigconv2 --pmc FETCH_SIZE -d gpurun_out/sptraffic/fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/sptraffic/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-include-regex k_bigconv2 --pmc WRITE_SIZE -d gpurun_out/sptraffic/write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/sptraffic/write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py gpurun_out/sptraffic "k_bigconv2[SP]" gpurun_out/r06_sp_traffic.json --dtype bf16x3 || exit $?
find gpurun_out/sptraffic -name "*.csv" -size +20M -delete
