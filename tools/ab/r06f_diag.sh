# which setting of test_gpu_knobs set1 breaks the aggregation: one variable at a time
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
C=tests/gpu_helpers/env_child.py
for kv in HBLS_SIG_CACHE=1024 HBLS_TA_JOINT=3 HBLS_TA_PAIR_MAX=100000 HBLS_WS_SETS=5 HBLS_GROUP_MAX=64 HBLS_FE_BATCH=4 HBLS_SLOT_MSM=64 HBLS_RLC_LANES=128; do
  env $kv timeout -k 10 120 python -u $C > $O/diag_r06f_$kv.json 2> $O/diag_r06f_$kv.err
  rc=$?
  echo "$kv rc=$rc"
  [ $rc -gt 1 ] && exit 1
done
exit 0
