# round 6: the C5 lines (1 % and 10 %) with their first-error figures
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--cpu-seconds 0 --callers 0 --key-tables 0 --host-api 0 --aggregate-verify 0"
timeout -k 10 600 python -u bench.py --workload c5 $Q > $O/bench_c5_r06c.json 2> $O/bench_c5_r06c.err || exit 1
timeout -k 10 600 python -u bench.py --workload c5 --bad-frac 0.10 $Q > $O/bench_c5_bad0.10_r06c.json 2> $O/bench_c5_bad0.10_r06c.err
