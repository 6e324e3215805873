# the C3 line at 5 / 20 / 40 timed steps (warm-up 2 / 5 / 5), one box: does a longer run lose throughput?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
for cfg in "5 2" "20 5" "40 5" "5 2" "20 5"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --steps $1 --warmup $2 $Q > $O/ab_r05ad_s$1_w$2_$(date +%s).json 2>> $O/ab_r05ad.err || exit 1
done
