# round-6 final-tree GPU record: GPU tests, smoke, the driver's bench command, then (second call) the profile
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r06fin} tools/gpu_check.sh ${STEPS:-test smoke driver}
