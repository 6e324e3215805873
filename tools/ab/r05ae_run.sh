# run-to-run variance of the C3 line at 20 steps, with the int_rates clock probe between runs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--steps 20 --warmup 5 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
X=tools/microbench/int_rates
for i in 1 2 3 4; do
  timeout -k 10 60 $X > $O/r05ae_probe_$i.txt 2>&1 || exit 1
  timeout -k 10 400 python -u bench.py $Q > $O/r05ae_bench_$i.json 2>> $O/r05ae.err || exit 1
done
timeout -k 10 60 $X > $O/r05ae_probe_5.txt 2>&1
