# GPU box: C3 bench with 1, 2 and 3 slots in flight, then a kernel trace at 2.  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
A="--workload c3 --steps 6 --warmup 2 --cpu-seconds 0 --callers 0 --aggregate-verify 0"
for k in 1 2 3; do
timeout -k 10 300 python -u bench.py $A --inflight $k > gpurun_out/inf_${TAG}_$k.json 2> gpurun_out/inf_${TAG}_$k.err || exit 1
done
bash tools/gpu_trace.sh $TAG $A --inflight 2
