cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_round6.sh r06z tests pftests smoke || exit $?
MNOR05=1 MSCENES="bunny:full bunny:primary soup:primary" MPOLICIES="lib nopred exact" bash tools/gpu_round6.sh r06z moving
