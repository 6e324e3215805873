# A/B: the slot stream's priority (C2, C3, C5)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
for rep in 1 2; do
  for pr in 0 -1; do
    for wl in c2 c3 c5; do
      HBLS_BENCH_STREAM_PRIO=$pr timeout -k 10 300 python -u bench.py --workload $wl $Q > $O/ab_r05j_${wl}_pr${pr}_$rep.json 2> $O/ab_r05j_${wl}_pr${pr}_$rep.err || exit 1
    done
  done
done
