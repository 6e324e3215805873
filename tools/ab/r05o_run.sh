# A/B: hardware queues x slots in flight (C2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
for cfg in "3 32" "3 24" "3 16" "4 16" "4 24" "4 8"; do
  set -- $cfg
  HBLS_WS_SETS=$1 HBLS_HW_QUEUES=$2 timeout -k 10 300 python -u bench.py --workload c2 --inflight $1 $Q > $O/ab_r05o_c2_if$1_q$2.json 2> $O/ab_r05o_c2_if$1_q$2.err || exit 1
done
