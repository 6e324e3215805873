# A/B: the MSM's weighing chunks of 16 buckets for small calls against 4 (HBLS_MSM_SMALL=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
Q="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 --key-tables 0"
bash tools/gpu.sh tests r05v "tests/test_gpu_scale.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_multi.py" || exit 1
for rep in 1 2; do
  for sm in 65536 0; do
    HBLS_MSM_SMALL=$sm timeout -k 10 300 python -u bench.py --workload c2 $Q > $O/ab_r05v_c2_msm${sm}_$rep.json 2> $O/ab_r05v_c2_msm${sm}_$rep.err || exit 1
  done
done
timeout -k 10 300 python -u bench.py --workload c3 $Q > $O/ab_r05v_c3.json 2> $O/ab_r05v_c3.err
