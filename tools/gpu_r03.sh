# GPU box (round 3): a pytest selection (files or -k), then optionally the default C3 bench.
#   $1 = tag, $2 = pytest args (quoted; "all" = every -m gpu test), $3 = bench (1/0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-q}
if [ "${2:-all}" = "all" ]; then SEL="tests"; else SEL="$2"; fi
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 150 --timeout-method thread --durations=15 > gpurun_out/tests_$TAG.log 2>&1 &&
if [ "${3:-0}" = "1" ]; then
timeout -k 10 400 python -u bench.py --workload c3 --steps 5 --warmup 2 --cpu-seconds 0 --callers 0 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err
fi
