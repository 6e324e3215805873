# round 6 first GPU pass: the review's robustness tests, the whole GPU suite, smoke, the C3 line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
bash tools/gpu.sh tests r06a_rob "tests/test_gpu_robustness.py" || exit 1
bash tools/gpu.sh tests r06a_all || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r06a.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3_r06a.json 2> $O/bench_c3_r06a.err
