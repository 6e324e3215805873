# Two-pass slot-wide MSM (the partials' entries sorted and summed beside the aggregation, the
# aggregates' added after it; HBLS_AB_MSM2=1) vs one pass after the groups' states (=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_scale.py tests/test_gpu_parity.py > $O/r05aq_tests.log 2>&1 || exit 1
Q="--cpu-seconds 0 --callers 0 --key-tables 0 --host-api 0 --aggregate-verify 0"
for rep in 1 2; do
  for e in 1 0; do
    HBLS_AB_MSM2=$e timeout -k 10 400 python -u bench.py --workload c2 --steps 20 --warmup 3 $Q > $O/ab_r05aq_c2_e${e}_$rep.json 2> $O/ab_r05aq_c2_e${e}_$rep.err || exit 1
  done
done
for e in 1 0; do
  HBLS_AB_MSM2=$e timeout -k 10 400 python -u bench.py --workload c3 --steps 20 --warmup 3 $Q > $O/ab_r05aq_c3_e$e.json 2> $O/ab_r05aq_c3_e$e.err || exit 1
done
timeout -k 10 400 python -u bench.py --workload c5 --steps 10 --warmup 2 $Q > $O/ab_r05aq_c5.json 2> $O/ab_r05aq_c5.err || exit 1
HBLS_ADAPTIVE=0 timeout -k 10 400 python -u bench.py --workload c5 --steps 3 --warmup 1 $Q > $O/ab_r05aq_c5_noadapt.json 2> $O/ab_r05aq_c5_noadapt.err || exit 1
HBLS_ADAPTIVE=0 timeout -k 10 400 python -u bench.py --workload c2 --bad-frac 0.01 --steps 5 --warmup 1 $Q > $O/ab_r05aq_c2bad_noadapt.json 2> $O/ab_r05aq_c2bad_noadapt.err
