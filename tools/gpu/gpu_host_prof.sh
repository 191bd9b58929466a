# host-side cost of the config-5 training step (tools/host_profile_step.py: cProfile over the timed steps only)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u tools/host_profile_step.py --dtype ${PROF_DT:-bf16} > gpurun_out/host_prof.txt 2>&1 || exit 3
head -3 gpurun_out/host_prof.txt
