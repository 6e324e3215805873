set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu.sh tests r06k "tests/test_gpu_multi.py"
