# round 6: the knob tests, the whole GPU suite, the C3 line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
bash tools/gpu.sh tests r06i_knobs "tests/test_gpu_knobs.py" || exit 1
bash tools/gpu.sh tests r06i_all || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3_r06i.json 2> $O/bench_c3_r06i.err
