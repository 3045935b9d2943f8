# round-6 final tree (merge beside the projection's last round): whole -m gpu suite, smoke, default bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PROF=0 bash tools/gpu_final.sh r06_final5
