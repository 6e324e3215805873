# round 6 final evidence on the final tree: the lines (C3/C2/C4/C5 + attack curve), the rocprofv3
# trace of the C3 line, PMC passes, and the torch.distributed.run launch path rehearsed (two ranks
# on the one GPU, --share-device)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
bash tools/gpu.sh lines r06m || exit 1
bash tools/gpu.sh attack r06m || exit 1
bash tools/gpu.sh trace r06m --steps 5 --warmup 2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 || exit 1
bash tools/gpu.sh pmc r06m || exit 1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --share-device 1 --workload c3 --validators 20000 --steps 3 --warmup 1 --cpu-seconds 0 --callers 0 \
  --aggregate-verify 0 --key-tables 0 --host-api 0 > $O/torchrun_rehearsal_r06m.json 2> $O/torchrun_rehearsal_r06m.err
