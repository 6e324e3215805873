# GPU box: one pytest selection + optional short C3 bench.  $1 = tag, $2 = pytest -k expr (or "all"), $3 = bench (1/0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-q}
K=${2:-all}
if [ "$K" = "all" ]; then KARG=""; else KARG="-k $K"; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $KARG > gpurun_out/tests_$TAG.log 2>&1 &&
if [ "${3:-1}" = "1" ]; then
timeout -k 10 400 python -u bench.py --workload c3 --steps 3 --warmup 1 --cpu-seconds 0 --callers 0 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err
fi
