# GPU box, end of round: GPU tests, smoke, the default bench line (C3), its rocprofv3 kernel trace,
# the PMC passes, and the C2 / C4 lines.  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-final}
B="$GRAFT_REPO_ROOT/bench.py"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err &&
timeout -k 10 300 python -u bench.py --workload c2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err &&
timeout -k 10 300 python -u bench.py --workload c4 --cpu-seconds 0 --callers 0 --aggregate-verify 0 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err &&
timeout -k 10 300 python -u bench.py --workload c5 --cpu-seconds 0 --callers 0 --key-tables 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 $B > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.err") &&
bash tools/gpu_pmc.sh $TAG
