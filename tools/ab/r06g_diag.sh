# test_gpu_knobs set1 with the aggregation detail, then set1 without one variable at a time
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
C=tests/gpu_helpers/env_child.py
S1="HBLS_WS_SETS=5 HBLS_COALESCE_US=2000 HBLS_COALESCE_MAX=3 HBLS_COALESCE_INFLIGHT=2 HBLS_SIG_CACHE=1024 HBLS_FE_BATCH=4 HBLS_SLOT_MSM=64 HBLS_SINGLE_MAX=1 HBLS_RLC_LANES=128 HBLS_TA_JOINT=3 HBLS_TA_PAIR_MAX=100000 HBLS_HASH_PAIR_MAX=100000 HBLS_HASH_ONE_LANE=100000 HBLS_FE18_MAX=100000 HBLS_GROUP_MAX=64"
env $S1 timeout -k 10 120 python -u $C > $O/diag_r06g_all.json 2> $O/diag_r06g_all.err
[ $? -gt 1 ] && exit 1
for drop in $S1; do
  rest=$(echo $S1 | tr ' ' '\n' | grep -v "^$drop\$" | tr '\n' ' ')
  env $rest timeout -k 10 120 python -u $C > "$O/diag_r06g_minus_$drop.json" 2> /dev/null
  rc=$?
  echo "minus $drop rc=$rc"
  [ $rc -gt 1 ] && exit 1
done
exit 0
