# GPU box: parity tests, slot bench and staged bench (no CPU baseline).  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-b2}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --mode staged > gpurun_out/bench_staged_$TAG.json 2> gpurun_out/bench_staged_$TAG.err
