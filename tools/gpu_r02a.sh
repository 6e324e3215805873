# GPU box, round 2 first call: Fp-product microbenchmark, parity tests, C3 bench, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02a}
timeout -k 10 120 ./tools/microbench/fpmul_variants 2048 > gpurun_out/fpmul_$TAG.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload c3 --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c3 --steps 2 --warmup 1 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json" 2>&1
