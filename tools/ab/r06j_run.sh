# A/B: signature-cache puts on per-context streams (product) vs one device put stream, on the
# concurrent-caller and host-buffer measurements of bench.py (same box, alternating, 3 reps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
A="--steps 3 --warmup 1 --cpu-seconds 0 --aggregate-verify 0 --key-tables 0 --callers 64 --callers-seconds 4"
for rep in 1 2 3; do
  for v in per_ctx one; do
    if [ $v = one ]; then export HBLS_LIBRARY=$GRAFT_REPO_ROOT/charon_amd/lib/variants/onestream/libhipbls.so; else unset HBLS_LIBRARY; fi
    timeout -k 10 300 python -u bench.py $A > $O/ab_r06j_${v}_$rep.json 2> $O/ab_r06j_${v}_$rep.err || exit 1
  done
done
