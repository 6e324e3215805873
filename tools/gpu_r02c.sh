# GPU box: parity tests, smoke, C3 bench with VerifyAggregate at scale.  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload c3 --steps 3 --warmup 1 --cpu-seconds 0 --callers 0 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err
