# Traffic-counter calibration on known bytes (tools/calib_traffic.py, csrc/calib.hip): FETCH_SIZE and
# WRITE_SIZE passes (separate, kernel-trace only) for C = 256 (tile 256, halo 5) and C = 128 (tile 512).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
for cfg in "256 256 5" "128 512 5"; do
  set -- $cfg
  tag=c$1
  A="--ld $1 --tile $2 --halo $3 --rows $((536870912 / $1))"
  rm -rf gpurun_out/calib/$tag
  timeout -s KILL 120 rocprofv3 --kernel-include-regex k_calib --pmc FETCH_SIZE -d gpurun_out/calib/$tag/fetch -o run --output-format csv -- python3 tools/calib_traffic.py run $A > gpurun_out/calib/$tag.fetch.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-include-regex k_calib --pmc WRITE_SIZE -d gpurun_out/calib/$tag/write -o run --output-format csv -- python3 tools/calib_traffic.py run $A > gpurun_out/calib/$tag.write.log 2>&1 || exit $?
  python3 tools/calib_traffic.py reduce gpurun_out/calib/$tag/fetch gpurun_out/calib/$tag/write gpurun_out/calib/$tag.json $A || exit $?
done
rocprofv3 -L > gpurun_out/calib/counters_list.txt 2>&1 || true
