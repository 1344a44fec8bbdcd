# Full GPU round: all -m gpu tests, then the profiling set (gpu_prof.sh).
cd $GRAFT_REPO_ROOT
bash scripts/gpu_tests.sh || exit $?
bash scripts/gpu_prof.sh
