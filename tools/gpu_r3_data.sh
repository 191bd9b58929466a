# Round-3 data batch: traffic calibration (modes 0-6), the dominant kernel's effective clock
# (GRBM_GUI_ACTIVE / 8 / duration, MI355X_MICROARCH.md DVFS), the config-5 bf16 train-step kernel stats.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_engine.py 13 0 8 16 24 > gpurun_out/ab_pf3.log 2>&1 || exit $?
head -5 gpurun_out/ab_pf3.log
bash tools/gpu_calib.sh > gpurun_out/calib.log 2>&1 || exit $?
tail -16 gpurun_out/calib.log
rm -rf gpurun_out/clk
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_bigconv --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/clk -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/clk.log 2>&1 || exit $?
echo "clock pass ok"
rm -rf gpurun_out/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o train --output-format csv -- python3 tools/bench_train_step.py --dtypes bf16 --steps 3 --warmup 1 > gpurun_out/prof_train.log 2>&1 || exit $?
tail -2 gpurun_out/prof_train.log | cut -c1-300
KERNEL=k_bigconv OUT=gpurun_out/traffic.json bash tools/gpu_traffic.sh > gpurun_out/traffic.log 2>&1 || exit $?
python3 tools/traffic_calibrated.py gpurun_out/traffic gpurun_out/calib/c256.json gpurun_out/calib/c128.json gpurun_out/traffic_calibrated.json > gpurun_out/traffic_calibrated.log 2>&1
tail -3 gpurun_out/traffic_calibrated.log
