# GPU box: the C3 bench under bench.py argument variants (one line each).  $1 = tag, then "ARGS" strings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
shift
k=0
for v in "$@"; do
  k=$((k+1))
  timeout -k 10 300 python -u bench.py --workload c3 --steps 4 --warmup 2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 $v > gpurun_out/arg_${TAG}_$k.json 2> gpurun_out/arg_${TAG}_$k.err || exit 1
  echo "$v" > gpurun_out/arg_${TAG}_$k.env
done
