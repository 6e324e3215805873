# HBLS_AB_TA bits (slots below ta_pair_max validators): 1 = k_ta_small's joint ladder on lane pairs,
# 2 = k_ta_stab and the pair ladders at one wave per SIMD (no scratch); 3 = both, 0 = neither
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_scale.py tests/test_gpu_parity.py > $O/r05ar_tests.log 2>&1 || exit 1
Q="--cpu-seconds 0 --callers 0 --key-tables 0 --host-api 0 --aggregate-verify 0"
for rep in 1 2; do
  for x in 3 0 1 2; do
    HBLS_AB_TA=$x timeout -k 10 400 python -u bench.py --workload c2 --steps 20 --warmup 3 $Q > $O/ab_r05ar_c2_x${x}_$rep.json 2> $O/ab_r05ar_c2_x${x}_$rep.err || exit 1
  done
done
HBLS_ADAPTIVE=0 timeout -k 10 400 python -u bench.py --workload c2 --bad-frac 0.01 --steps 5 --warmup 1 $Q > $O/ab_r05ar_c2bad_noadapt.json 2> $O/ab_r05ar_c2bad_noadapt.err
