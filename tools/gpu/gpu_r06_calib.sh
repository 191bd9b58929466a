# Round 6: traffic-counter calibration for every k_bigconv access pattern of the headline decode:
# window rows of 64, 128, 256, 512 and 1024 channels (modes 0-6), and the polyphase upsamplers' strided epilogue
# stores / residual loads (modes 7 / 8) at (Cout, up) = (256, 10), (128, 5), (64, 3).  FETCH_SIZE and WRITE_SIZE in
# separate passes, kernel-trace only; rows a multiple of 960 (the upsampling factors x 32)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/calib6
for cfg in "1024 256 5" "512 256 1" "256 256 10" "128 512 5" "64 512 3"; do
  set -- $cfg
  tag=c$1
  rows=$(( (536870912 / $1) / 960 * 960 ))
  A="--ld $1 --tile $2 --halo $3 --rows $rows"
  rm -rf gpurun_out/calib6/$tag
  timeout -s KILL 120 rocprofv3 --kernel-include-regex k_calib --pmc FETCH_SIZE -d gpurun_out/calib6/$tag/fetch -o run --output-format csv -- python3 tools/calib_traffic.py run $A > gpurun_out/calib6/$tag.fetch.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-include-regex k_calib --pmc WRITE_SIZE -d gpurun_out/calib6/$tag/write -o run --output-format csv -- python3 tools/calib_traffic.py run $A > gpurun_out/calib6/$tag.write.log 2>&1 || exit $?
  python3 tools/calib_traffic.py reduce gpurun_out/calib6/$tag/fetch gpurun_out/calib6/$tag/write gpurun_out/calib6/$tag.json $A > gpurun_out/calib6/$tag.txt 2>&1 || exit $?
  cat gpurun_out/calib6/$tag.txt
  rm -rf gpurun_out/calib6/$tag
done
# the family's own FETCH / WRITE passes over one headline step (each launch alone: noise branches off)
export BENCH_ARGS="--no-parity-mode --no-accuracy-mode --no-e2e"
export STTS_OPTS=24=0
KERNEL=k_bigconv OUT=gpurun_out/r06_traffic_raw.json bash tools/gpu/gpu_traffic.sh > gpurun_out/r06_traffic.log 2>&1 || exit $?
echo traffic ok
