# RCCL plumbing smoke at world size 1 (tools/rccl_smoke.py)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 180 python -u tools/rccl_smoke.py > gpurun_out/rccl_smoke.log 2>&1 || exit $?
tail -4 gpurun_out/rccl_smoke.log
