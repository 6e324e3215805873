# slots in flight 3 / 4 / 5 with the host-call contexts' streams created lazily (fewer idle streams holding hardware queues)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
for rep in 1 2; do
  for k in 3 4 5; do
    for wl in c2 c3; do
      HBLS_WS_SETS=$k timeout -k 10 300 python -u bench.py --workload $wl --inflight $k $Q > $O/ab_r05aa_${wl}_if${k}_$rep.json 2> $O/ab_r05aa_${wl}_if${k}_$rep.err || exit 1
    done
  done
done
