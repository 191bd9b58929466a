# Round-2 PMC passes of the bigconv engines over one bench step + the HBM traffic JSON bench.py
# picks up as roofline.traffic (kernel name 'k_bigconv' matches both bigconv.hip and bigconv2.hip)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export KREGEX=k_bigconv
export BENCH_ARGS="--no-parity-mode --no-e2e"
bash tools/gpu_pmc.sh > gpurun_out/pmc_r02.log 2>&1 || exit $?
python3 tools/analyze_pmc.py gpurun_out/pmc > gpurun_out/pmc_bigconv_r02.txt 2>&1 || exit $?
KERNEL=k_bigconv OUT=gpurun_out/r02_traffic.json bash tools/gpu_traffic.sh > gpurun_out/traffic_r02.log 2>&1 || exit $?
