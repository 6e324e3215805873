# Slots in flight with paced enqueue: 3 (default) vs 4 workspace sets / slots, C3 and C2, two reps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
Q="--cpu-seconds 0 --callers 0 --key-tables 0 --host-api 0 --aggregate-verify 0"
for rep in 1 2; do
  for f in 3 4; do
    HBLS_WS_SETS=$f timeout -k 10 400 python -u bench.py --workload c3 --inflight $f --steps 20 --warmup 3 $Q > $O/ab_r05as_c3_f${f}_$rep.json 2> $O/ab_r05as_c3_f${f}_$rep.err || exit 1
    HBLS_WS_SETS=$f timeout -k 10 400 python -u bench.py --workload c2 --inflight $f --steps 20 --warmup 3 $Q > $O/ab_r05as_c2_f${f}_$rep.json 2> $O/ab_r05as_c2_f${f}_$rep.err || exit 1
  done
done
