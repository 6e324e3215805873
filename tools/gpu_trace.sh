# GPU box: parity tests, slot bench, and a kernel-trace of the slot bench (timeline).  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-tr}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json" 2>&1
