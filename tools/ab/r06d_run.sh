set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu.sh tests r06d "tests/test_signing_roots.py tests/test_go_shim.py tests/test_library_abi.py"
