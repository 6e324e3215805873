# C2 kernel trace (10 slots) for the timeline of a small slot; C2 line alongside
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
B=$GRAFT_REPO_ROOT/bench.py
A="--workload c2 --steps 10 --warmup 2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 --host-api 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r05an_c2 -o run --output-format csv -- python3 $B $A \
  > $O/bench_prof_r05an_c2.json 2> $O/bench_prof_r05an_c2.err
