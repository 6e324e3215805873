# GPU box: effective shader clock per kernel (GRBM_GUI_ACTIVE / duration) over a staged C3 slot.  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
B="$GRAFT_REPO_ROOT/bench.py"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_INSTS_VALU -d "$GRAFT_REPO_ROOT/gpurun_out/clk_$TAG" -o run --output-format csv -- python3 $B --workload c3 --steps 1 --warmup 0 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --mode staged --inflight 1 > "$GRAFT_REPO_ROOT/gpurun_out/clk_$TAG.log" 2>&1
