# GPU box: C3 bench (staged, one slot in flight: clean per-kernel times; then slot mode, two in
# flight) for the product library and each tuning variant under charon_amd/lib/variants/.
# $1 = tag, $2.. = variant names
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
A="--workload c3 --steps 4 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0"
for v in base "$@"; do
  if [ "$v" = base ]; then LIBV=""; else LIBV=charon_amd/lib/variants/$v/libhipbls.so; fi
  HBLS_LIBRARY=$LIBV timeout -k 10 300 python -u bench.py $A --mode staged --inflight 1 > gpurun_out/var_${TAG}_${v}_staged.json 2> gpurun_out/var_${TAG}_${v}_staged.err || exit 1
  HBLS_LIBRARY=$LIBV timeout -k 10 300 python -u bench.py $A > gpurun_out/var_${TAG}_${v}_slot.json 2> gpurun_out/var_${TAG}_${v}_slot.err || exit 1
done
