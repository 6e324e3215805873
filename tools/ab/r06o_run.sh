# the final tree as the driver runs it at round end: the GPU suite, then smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_r06o.txt 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke_r06o.txt 2>&1
