# stdout of the bench is exactly the one JSON line: the driver's N=1 command, the torch.distributed.run
# launch (two ranks rehearsed on the one GPU) and bench.py's own launcher
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
A="--workload c3 --validators 20000 --steps 3 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 --host-api 0"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/n1_r06n.out 2> $O/n1_r06n.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --share-device 1 $A > $O/torchrun_r06n.out 2> $O/torchrun_r06n.err &&
timeout -k 10 300 python bench.py --gpus 2 --share-device 1 $A > $O/selflaunch_r06n.out 2> $O/selflaunch_r06n.err &&
wc -l $O/n1_r06n.out $O/torchrun_r06n.out $O/selflaunch_r06n.out
