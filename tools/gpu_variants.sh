# GPU box: C3 bench for the product library and each tuning variant under charon_amd/lib/variants/.
# $1 = tag, $2.. = variant names
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0 > gpurun_out/var_${TAG}_base.json 2> gpurun_out/var_${TAG}_base.err || exit 1
for v in "$@"; do
  HBLS_LIBRARY=charon_amd/lib/variants/$v/libhipbls.so timeout -k 10 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0 > gpurun_out/var_${TAG}_$v.json 2> gpurun_out/var_${TAG}_$v.err || exit 1
done
