# A/B: hardware queues x slots in flight (C2, C3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
for wl in c2 c3; do
for cfg in "3 8" "3 12" "4 8" "4 12" "5 8" "6 8" "3 32"; do
  set -- $cfg
  HBLS_WS_SETS=$1 HBLS_HW_QUEUES=$2 timeout -k 10 300 python -u bench.py --workload $wl --inflight $1 $Q > $O/ab_r05p_${wl}_if$1_q$2.json 2> $O/ab_r05p_${wl}_if$1_q$2.err || exit 1
done
done
