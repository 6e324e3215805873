# GPU box: C3 and C2, default streams vs one stream per slot (HBLS_SERIAL_SLOT), 3 / 4 in flight.  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
for wl in c3 c2; do
  for v in "0 3" "1 3" "1 4" "0 3" "1 4"; do
    set -- $v
    HBLS_SERIAL_SLOT=$1 timeout -k 10 300 python -u bench.py --workload $wl --steps 6 --warmup 2 --inflight $2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 > gpurun_out/ser_${TAG}_${wl}_$1_$2.json 2> gpurun_out/ser_${TAG}_${wl}_$1_$2.err || exit 1
    echo "serial=$1 inflight=$2 $(python3 tools/bsum.py gpurun_out/ser_${TAG}_${wl}_$1_$2.json | head -1)" >> gpurun_out/ser_${TAG}.txt
  done
done
