# round 6: whole GPU suite (C client, two-rank rehearsal included), smoke, the driver's C3 command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
bash tools/gpu.sh tests r06l || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r06l.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3_r06l.json 2> $O/bench_c3_r06l.err
