# GPU box: GPU tests, then the C3 bench (staged + slot) with each environment setting given.
# $1 = tag, $2.. = "NAME=VALUE" settings ("-" = none)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
A="--workload c3 --steps 4 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit 1
k=0
for e in "$@"; do
  k=$((k+1))
  if [ "$e" = "-" ]; then E=""; else E="$e"; fi
  env $E timeout -k 10 300 python -u bench.py $A --mode staged --inflight 1 > gpurun_out/env_${TAG}_${k}_staged.json 2> gpurun_out/env_${TAG}_${k}_staged.err || exit 1
  env $E timeout -k 10 300 python -u bench.py $A > gpurun_out/env_${TAG}_${k}_slot.json 2> gpurun_out/env_${TAG}_${k}_slot.err || exit 1
done
