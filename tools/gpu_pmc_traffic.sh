# GPU box: HBM traffic of every kernel of one C2 bench step, two PMC passes (FETCH_SIZE, WRITE_SIZE).  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-traffic}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch_$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 --steps 1 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch_$TAG.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write_$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 --steps 1 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_write_$TAG.log" 2>&1
