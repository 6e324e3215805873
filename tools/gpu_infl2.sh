# GPU box: C2 and C3 lines with 3 and 4 slots in flight (same box).  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
for wl in c2 c3; do
  for k in 3 4 3 4; do
    timeout -k 10 300 python -u bench.py --workload $wl --steps 6 --warmup 2 --inflight $k --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 > gpurun_out/if_${TAG}_${wl}_$k.json 2> gpurun_out/if_${TAG}_${wl}_$k.err || exit 1
    python3 tools/bsum.py gpurun_out/if_${TAG}_${wl}_$k.json | head -1 >> gpurun_out/if_${TAG}.txt
  done
done
