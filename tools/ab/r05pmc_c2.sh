# C2: VALU instructions per slot (one PMC pass over a 1-step bench run) and the GPU suite's scale tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
bash tools/gpu.sh tests r05t2 tests/test_gpu_scale.py || exit 1
cd /tmp && export TMPDIR=/tmp
A="--workload c2 --steps 1 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 --host-api 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/pmc_c2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $A > $O/pmc_c2.log 2>&1
