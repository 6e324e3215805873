# GPU box: list counters, then one PMC pass over a short bench run.  $1 = tag, $2.. = counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/counters_list.txt" 2>&1
timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 --steps 1 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG.log" 2>&1
