# GPU box: parity tests (incl. scale/adversarial), smoke, C3 + C2 bench, kernel-trace summary.  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload c3 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err &&
timeout -k 10 300 python -u bench.py --workload c2 --steps 5 --warmup 2 --cpu-seconds 0 --callers 0 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c3 --steps 2 --warmup 1 --cpu-seconds 0 --callers 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json" 2>&1
