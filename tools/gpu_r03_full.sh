# GPU box (round 3): the whole -m gpu suite, smoke(), then tools/gpu_r03_prof.sh (C3 bench line,
# rocprofv3 trace, C2/C4/C5 lines).  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || exit 1
bash tools/gpu_r03_prof.sh "$TAG" ""
