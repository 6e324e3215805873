# round 6 evidence pass on the current tree: smoke, the C3/C2/C4/C5 lines, the attack curve, the
# rocprofv3 trace of the C3 line, PMC passes (pmc_traffic.json), one slot's kernel timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r06h.log 2>&1 || exit 1
bash tools/gpu.sh lines r06h || exit 1
bash tools/gpu.sh attack r06h || exit 1
bash tools/gpu.sh trace r06h --steps 5 --warmup 2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 || exit 1
bash tools/gpu.sh pmc r06h
