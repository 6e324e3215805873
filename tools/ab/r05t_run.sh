# A/B: the aggregation's [s] ladder on lane pairs (default at C2) against one lane (HBLS_TA_PAIR_MAX=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
bash tools/gpu.sh tests r05t "tests/test_gpu_scale.py tests/test_gpu_configs.py tests/test_gpu_parity.py" || exit 1
for rep in 1 2; do
  for pm in 16384 0; do
    HBLS_TA_PAIR_MAX=$pm timeout -k 10 300 python -u bench.py --workload c2 $Q > $O/ab_r05t_c2_ta${pm}_$rep.json 2> $O/ab_r05t_c2_ta${pm}_$rep.err || exit 1
  done
done
