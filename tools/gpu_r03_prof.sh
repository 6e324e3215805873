# GPU box (round 3): the default bench line (C3), a rocprofv3 kernel trace of a short C3 run (last
# slot = the serialised roofline slot), and the C2 / C4 / C5 lines.  $1 = tag, $2 = pytest -k expr
# to run first ("" = none)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-prof}
B="$GRAFT_REPO_ROOT/bench.py"
if [ -n "$2" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "$2" > gpurun_out/tests_$TAG.log 2>&1 || exit 1
fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 $B --steps 2 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 --host-api 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.err") &&
timeout -k 10 300 python -u bench.py --workload c2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err &&
timeout -k 10 300 python -u bench.py --workload c4 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err &&
timeout -k 10 300 python -u bench.py --workload c5 --cpu-seconds 0 --callers 0 --key-tables 0 --host-api 0 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err
