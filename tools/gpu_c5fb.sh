# GPU box: GPU tests, then the C5 line under fallback batch sizes.  $1 = tag
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit 1
for fb in 64 8 4 16; do
  HBLS_FALLBACK_BATCH=$fb timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 > gpurun_out/c5fb_${TAG}_$fb.json 2> gpurun_out/c5fb_${TAG}_$fb.err || exit 1
done
