# GPU box: one workload's bench line under environment variants.  $1 = tag, $2 = workload, then "NAME=VAL ..." strings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
WL=$2
shift 2
k=0
for v in "$@"; do
  k=$((k+1))
  env $v timeout -k 10 300 python -u bench.py --workload $WL --steps 5 --warmup 2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 > gpurun_out/wl_${TAG}_$k.json 2> gpurun_out/wl_${TAG}_$k.err || exit 1
  echo "$v" > gpurun_out/wl_${TAG}_$k.env
done
