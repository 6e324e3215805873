# A/B: the bench's timed region with and without per-launch event instrumentation (C2, C3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
for rep in 1 2; do
  for ev in 0 1; do
    for wl in c2 c3; do
      HBLS_BENCH_TIMED_EVENTS=$ev timeout -k 10 300 python -u bench.py --workload $wl $Q > $O/ab_r05i_${wl}_ev${ev}_$rep.json 2> $O/ab_r05i_${wl}_ev${ev}_$rep.err || exit 1
    done
  done
done
