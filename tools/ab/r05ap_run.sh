# C2 at 20 steps / 3 warmup (the 5-step default line is mostly pipeline fill and drain at 8-10 ms per slot), twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
Q="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0"
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py --workload c2 --steps 20 --warmup 3 $Q > $O/bench_c2_r05ap_$rep.json 2> $O/bench_c2_r05ap_$rep.err || exit 1
done
