# round 6: first-error mode tests, the C5 line with its first-error figure
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
bash tools/gpu.sh tests r06b_first "tests/test_gpu_first_error.py tests/test_gpu_robustness.py" || exit 1
timeout -k 10 600 python -u bench.py --workload c5 --cpu-seconds 0 --callers 0 --key-tables 0 --host-api 0 --aggregate-verify 0 > $O/bench_c5_r06b.json 2> $O/bench_c5_r06b.err || exit 1
timeout -k 10 600 python -u bench.py --workload c5 --bad-frac 0.10 --cpu-seconds 0 --callers 0 --key-tables 0 --host-api 0 --aggregate-verify 0 > $O/bench_c5_bad0.10_r06b.json 2> $O/bench_c5_bad0.10_r06b.err
