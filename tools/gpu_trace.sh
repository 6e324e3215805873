# GPU box: kernel trace of a short C3 bench run.  $1 = tag, rest = bench args
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
B="$GRAFT_REPO_ROOT/bench.py"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/trace_$TAG" -o run --output-format csv -- python3 $B "$@" > "$GRAFT_REPO_ROOT/gpurun_out/trace_$TAG.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/trace_$TAG.err"
