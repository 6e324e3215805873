# the C3 line at 20 steps with paced slots (the default), four runs, then the driver's exact command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--steps 20 --warmup 5 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
for i in 1 2 3 4; do
  timeout -k 10 400 python -u bench.py $Q > $O/r05ag_paced_$i.json 2>> $O/r05ag.err || exit 1
done
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/r05ag_driverlike.json 2>> $O/r05ag.err
