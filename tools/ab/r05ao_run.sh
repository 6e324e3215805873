# HBLS_AB_X bits: 1 = the aggregation's index-only split (k_ta_sprep) before the members are decompressed,
# 2 = the MSM's bucket counters zeroed before the check's wait; 3 = both (the change), 0 = neither
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_scale.py tests/test_gpu_parity.py > $O/r05ao_tests.log 2>&1 || exit 1
Q="--cpu-seconds 0 --callers 0 --key-tables 0 --host-api 0 --aggregate-verify 0"
for rep in 1 2; do
  for x in 3 0 1 2; do
    HBLS_AB_X=$x timeout -k 10 400 python -u bench.py --workload c2 --steps 20 --warmup 3 $Q > $O/ab_r05ao_c2_x${x}_$rep.json 2> $O/ab_r05ao_c2_x${x}_$rep.err || exit 1
  done
  for x in 3 0; do
    HBLS_AB_X=$x timeout -k 10 400 python -u bench.py --workload c3 --steps 20 --warmup 3 $Q > $O/ab_r05ao_c3_x${x}_$rep.json 2> $O/ab_r05ao_c3_x${x}_$rep.err || exit 1
  done
done
