# Round 6: resconv tests after the interleaved-epilogue default (STTS_OPT_RCPP 3), then the decoder suites
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_decoder.py tests/test_gpu_edge.py -m gpu -q -rfE --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_iltest.log 2>&1
rc=$?; tail -6 gpurun_out/r06_iltest.log; exit $rc
