# concurrent single-item callers: coalescing window 200 (default) / 500 / 1000 us, C2 data (the callers leg only matters)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--steps 2 --warmup 1 --cpu-seconds 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
for rep in 1 2; do
  for us in 200 500 1000; do
    HBLS_COALESCE_US=$us timeout -k 10 300 python -u bench.py --workload c2 $Q > $O/ab_r05ac_us${us}_$rep.json 2> $O/ab_r05ac_us${us}_$rep.err || exit 1
  done
done
