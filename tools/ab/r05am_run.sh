# The partials' key-side combination beside the signatures' subgroup checks (e1) vs after them (e0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_scale.py tests/test_gpu_parity.py > $O/r05am_tests.log 2>&1 || exit 1
Q="--cpu-seconds 0 --callers 0 --key-tables 0 --host-api 0 --aggregate-verify 0"
for rep in 1 2; do
  for e in 1 0; do
    for wl in c2 c3; do
      HBLS_AB_PK_EARLY=$e timeout -k 10 400 python -u bench.py --workload $wl --steps 20 --warmup 3 $Q > $O/ab_r05am_${wl}_e${e}_$rep.json 2> $O/ab_r05am_${wl}_e${e}_$rep.err || exit 1
    done
  done
done
HBLS_AB_PK_EARLY=1 timeout -k 10 400 python -u bench.py --workload c5 --steps 10 --warmup 2 $Q > $O/ab_r05am_c5_e1.json 2> $O/ab_r05am_c5_e1.err
for a in 0 1; do
  HBLS_ADAPTIVE=$a timeout -k 10 400 python -u bench.py --workload c2 --bad-frac 0.01 --steps 5 --warmup 1 $Q > $O/ab_r05am_c2bad_adapt$a.json 2> $O/ab_r05am_c2bad_adapt$a.err || exit 1
done
