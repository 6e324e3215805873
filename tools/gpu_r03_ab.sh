# GPU box (round 3): GPU tests (pytest -k $2, "all" = every test), then C2 / C3 bench lines under
# environment variants.  $1 = tag; then "WORKLOAD:NAME=VAL ...|bench args" strings ("-" = no variables)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
SEL=$2
shift 2
if [ "$SEL" = "all" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit 1
elif [ -n "$SEL" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "$SEL" > gpurun_out/tests_$TAG.log 2>&1 || exit 1
fi
k=0
for v in "$@"; do
  k=$((k+1))
  wl=${v%%:*}
  rest=${v#*:}
  vars=${rest%%|*}
  extra=""
  [ "$rest" != "$vars" ] && extra=${rest#*|}
  [ "$vars" = "-" ] && vars=""
  env $vars timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 --host-api 0 $extra > gpurun_out/ab_${TAG}_$k.json 2> gpurun_out/ab_${TAG}_$k.err || exit 1
  echo "$v" > gpurun_out/ab_${TAG}_$k.env
done
