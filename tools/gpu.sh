# GPU box driver (run through gpurun from the repo root):  bash tools/gpu.sh <what> <tag> [args]
#   tests  TAG [pytest selection]   -m gpu tests (default: all of tests/), log gpurun_out/tests_TAG.log
#   bench  TAG WORKLOAD [bench args] one bench.py line -> gpurun_out/bench_WORKLOAD_TAG.json
#   lines  TAG                      C3 default line, then the C2 / C4 / C5 lines
#   trace  TAG [bench args]         rocprofv3 kernel trace + stats of a bench run
#   pmc    TAG                      kernel trace + SQ / FETCH_SIZE / WRITE_SIZE passes over one C3 slot
#   final  TAG                      tests, smoke, lines, trace of the default C3 line, pmc
#   single TAG [calls]              kernel trace of single-item Verify calls (tools/diag_single.py)
#   peak   TAG                      int_rates microbenchmark: plain, kernel trace, PMC pass (the peak)
#   attack TAG                      C5 at 5 % and 10 % corrupted partials (the 1 % point is in `lines`)
# Every GPU step has its own time limit and the steps are chained with &&: the first failure,
# abort or time-out ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
WHAT=$1
TAG=${2:-x}
shift 2
B="$GRAFT_REPO_ROOT/bench.py"
O="$GRAFT_REPO_ROOT/gpurun_out"
QUIET="--cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0"

tests() {
  timeout -k 10 900 python -u -m pytest ${1:-tests} -m gpu -x -v --timeout 300 --timeout-method thread --durations=20 \
    > "$O/tests_$TAG.log" 2>&1
}
smoke() {
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$TAG.log" 2>&1
}
bench() {
  local wl=$1
  shift
  timeout -k 10 600 python -u bench.py --workload "$wl" "$@" > "$O/bench_${wl}_$TAG.json" 2> "$O/bench_${wl}_$TAG.err"
}
lines() {
  bench c3 &&
  bench c2 $QUIET --steps 20 --warmup 3 &&
  bench c4 $QUIET &&
  bench c5 --cpu-seconds 0 --callers 0 --key-tables 0 --host-api 0
}
trace() {
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_$TAG" -o run --output-format csv -- python3 "$B" "$@" \
     > "$O/bench_prof_$TAG.json" 2> "$O/bench_prof_$TAG.err")
}
pmc() {
  local P="$O/pmc_$TAG"
  local A="--workload c3 --steps 1 --warmup 1 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --key-tables 0 --host-api 0"
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/trace" -o run --output-format csv -- python3 "$B" $A > "$P.trace.log" 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d "$P/sq" -o run --output-format csv -- python3 "$B" $A > "$P.sq.log" 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$P/fetch" -o run --output-format csv -- python3 "$B" $A > "$P.fetch.log" 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$P/write" -o run --output-format csv -- python3 "$B" $A > "$P.write.log" 2>&1)
}
peak() {  # the roofline peak pinned by counters (tools/microbench/int_rates_pmc.py)
  local P="$O/peak_$TAG"
  local X="$GRAFT_REPO_ROOT/tools/microbench/int_rates"
  mkdir -p "$P"
  timeout -k 10 120 "$X" > "$P/int_rates_plain.txt" 2>&1 &&
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 120 rocprofv3 --kernel-trace -d "$P/trace" -o run --output-format csv -- "$X" > "$P/int_rates.txt" 2>&1 &&
   timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$P/pmc" -o run \
     --output-format csv -- "$X" > "$P/pmc.log" 2>&1)
}
attack() {
  local f
  for f in 0.05 0.10; do
    timeout -k 10 600 python -u bench.py --workload c5 --bad-frac $f --cpu-seconds 0 --callers 0 --key-tables 0 \
      --host-api 0 > "$O/bench_c5_bad${f}_$TAG.json" 2> "$O/bench_c5_bad${f}_$TAG.err" || return 1
  done
}
single() {
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/single_$TAG" -o run --output-format csv -- python3 \
     "$GRAFT_REPO_ROOT/tools/diag_single.py" "${1:-8}" > "$O/single_$TAG.log" 2>&1)
}

# A/B of library builds on one box (HBLS_LIBRARY): ab TAG WORKLOAD label=path ... ; alternates
# through the list twice, one bench line each (bench args from $AB_ARGS)
ab() {
  local wl=$1
  shift
  for rep in 1 2; do
    for spec in "$@"; do
      local lab=${spec%%=*} lib=${spec#*=}
      HBLS_LIBRARY="$lib" timeout -k 10 400 python -u bench.py --workload "$wl" ${AB_ARGS:-$QUIET --key-tables 0} \
        > "$O/ab_${TAG}_${wl}_${lab}_$rep.json" 2> "$O/ab_${TAG}_${wl}_${lab}_$rep.err" || return 1
    done
  done
}

case "$WHAT" in
  tests) tests "$@" ;;
  bench) bench "$@" ;;
  lines) lines ;;
  trace) trace "$@" ;;
  pmc) pmc ;;
  final) tests && smoke && lines && trace --steps 5 --warmup 2 --cpu-seconds 0 --callers 0 --aggregate-verify 0 --host-api 0 && pmc ;;
  ab) ab "$@" ;;
  single) single "$@" ;;
  peak) peak ;;
  attack) attack ;;
  *) echo "usage: bash tools/gpu.sh tests|bench|lines|trace|pmc|final|ab|single|peak|attack TAG [args]" >&2; exit 2 ;;
esac
