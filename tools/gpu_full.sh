# GPU box: parity tests, smoke, default bench (with CPU baseline), staged bench, kernel-trace summary.  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-full}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --mode staged > gpurun_out/bench_staged_$TAG.json 2> gpurun_out/bench_staged_$TAG.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json" 2>&1
