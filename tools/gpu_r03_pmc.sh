# GPU box (round 3): kernel trace + three PMC passes (SQ counters, FETCH_SIZE, WRITE_SIZE) over one
# C3 slot, then a kernel trace of one C5 step (the fallback path).  $1 = tag.  Each pass is its own
# rocprofv3 run (no trace domains with --pmc).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-pmc}
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG"
B="$GRAFT_REPO_ROOT/bench.py"
ARGS="--workload c3 --steps 1 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 --host-api 0"
C5="--workload c5 --steps 1 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 --host-api 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $B $ARGS > "$OUT.trace.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d "$OUT/sq" -o run --output-format csv -- python3 $B $ARGS > "$OUT.sq.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $B $ARGS > "$OUT.fetch.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $B $ARGS > "$OUT.write.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c5trace" -o run --output-format csv -- python3 $B $C5 > "$OUT.c5trace.log" 2>&1
