# paced slots (default) against every slot up front (HBLS_BENCH_PACE=0): C2, C4, C5 lines, alternating, two runs each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
for rep in 1 2; do
  for wl in c2 c4 c5; do
    for p in 1 0; do
      HBLS_BENCH_PACE=$p timeout -k 10 400 python -u bench.py --workload $wl $Q > $O/ab_r05ah_${wl}_pace${p}_$rep.json 2>> $O/ab_r05ah.err || exit 1
    done
  done
done
