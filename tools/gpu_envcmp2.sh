# GPU box: slot-mode bench of a workload with each environment setting.  $1 = tag, $2 = workload,
# $3.. = "NAME=VALUE" settings ("-" = none)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; W=$2; shift; shift
A="--workload $W --steps 5 --warmup 2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0"
k=0
for e in "$@"; do
  k=$((k+1))
  if [ "$e" = "-" ]; then E=""; else E="$e"; fi
  env $E timeout -k 10 300 python -u bench.py $A > gpurun_out/e2_${TAG}_${W}_${k}.json 2> gpurun_out/e2_${TAG}_${W}_${k}.err || exit 1
done
