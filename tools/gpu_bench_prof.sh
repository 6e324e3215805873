# GPU box: smoke, bench (default C2 workload) and a rocprofv3 kernel-trace summary of the same bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json" 2>&1
