set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
bash tools/gpu.sh tests r05h "tests/test_gpu_sigcache.py tests/test_gpu_configs.py" &&
HBLS_DEC_PAIR_MAX=1000000 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sigcache.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_r05h_pair.log 2>&1 &&
HBLS_HOST_TIMING=1 bash tools/gpu.sh bench r05h c3 --cpu-seconds 0 --aggregate-verify 0 --callers 0 --key-tables 0 &&
for rep in 1 2; do
  for pm in 0 65536; do
    HBLS_DEC_PAIR_MAX=$pm timeout -k 10 300 python -u bench.py --workload c2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0 > $O/ab_r05h_c2_pm${pm}_$rep.json 2> $O/ab_r05h_c2_pm${pm}_$rep.err || exit 1
  done
done &&
bash tools/gpu.sh trace r05h_c2 --workload c2 --steps 5 --warmup 2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0
