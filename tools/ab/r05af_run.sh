# run-to-run spread of the C3 line at 20 steps: every slot enqueued up front (pace0) or each after the one
# before it on its stream completed (pace1), alternating, four runs each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--steps 20 --warmup 5 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
for i in 1 2 3 4; do
  for p in 0 1; do
    HBLS_BENCH_PACE=$p timeout -k 10 400 python -u bench.py $Q > $O/ab_r05af_pace${p}_$i.json 2>> $O/ab_r05af.err || exit 1
  done
done
