#!/bin/bash
# One entry point for every GPU-box job (run through gpurun); each GPU step has its own time limit, steps chain
# with &&-semantics (the script stops at the first failure), output lands under gpurun_out/.
#
#   scripts/gpu.sh tests [pytest -k expr]        GPU test suite (optionally filtered)
#   scripts/gpu.sh full                           GPU suite + smoke + default bench (as the driver runs them)
#   scripts/gpu.sh bench <name> [bench args]      one bench.py JSON line -> gpurun_out/benches/<name>.log
#   scripts/gpu.sh matrix                         the BASELINE config matrix (scripts/bench_matrix.sh)
#   scripts/gpu.sh profile <tag> [bench args]     rocprofv3 kernel trace + stats summary (scripts/profile_one.sh)
#   scripts/gpu.sh ab <VAR> <v1,v2,..> [bench args]  the same bench under each value of an env knob
#   scripts/gpu.sh pmc <CTR,CTR,..> [bench args]  one rocprofv3 counter pass (stats only, no trace domains)
#   scripts/gpu.sh py <script.py> [args]          a measurement script (scripts/bench_*.py), stdout -> jsonl
# Several jobs: scripts/gpu.sh "tests prefill" "bench b32 --steps 3"   (each quoted job in order)
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/benches

job() {
  local kind=$1; shift
  case "$kind" in
    tests)
      timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -rf -x --timeout 150 --timeout-method thread \
        ${1:+-k "$*"} > gpurun_out/gpu_tests.log 2>&1
      local rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || tail -60 gpurun_out/gpu_tests.log; return $rc ;;
    full)
      job tests || return 1
      timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 \
        || { tail -n 20 gpurun_out/smoke.log; return 2; }
      tail -n 1 gpurun_out/smoke.log
      job bench default ;;
    bench)
      local name=$1; shift
      timeout -k 10 500 python -u bench.py "$@" > gpurun_out/benches/$name.log 2>&1
      local rc=$?; tail -1 gpurun_out/benches/$name.log; [ $rc -eq 0 ] || tail -30 gpurun_out/benches/$name.log; return $rc ;;
    matrix) bash scripts/bench_matrix.sh ;;
    profile) bash scripts/profile_one.sh "$@" ;;
    ab)
      local var=$1 vals=$2; shift 2
      for v in ${vals//,/ }; do
        env "$var=$v" timeout -k 10 500 python -u bench.py "$@" > gpurun_out/benches/ab_${var}_$v.log 2>&1 \
          || { tail -30 gpurun_out/benches/ab_${var}_$v.log; return 3; }
        echo "$var=$v $(tail -1 gpurun_out/benches/ab_${var}_$v.log | cut -c1-400)"
      done ;;
    pmc)
      local ctr=$1; shift
      mkdir -p gpurun_out/pmc
      timeout -s KILL 300 rocprofv3 --pmc ${ctr//,/ } --kernel-trace --stats --output-format csv \
        -d gpurun_out/pmc/${ctr//,/_} -o run -- python3 bench.py "$@" > gpurun_out/pmc/${ctr//,/_}.log 2>&1
      local rc=$?; find gpurun_out/pmc/${ctr//,/_} -name "*kernel_trace.csv" -delete; return $rc ;;
    py)
      local script=$1; shift
      local out=gpurun_out/$(basename "$script" .py).jsonl
      timeout -k 10 600 python -u "$script" "$@" > "$out" 2> "${out%.jsonl}.err"
      local rc=$?; tail -20 "$out"; [ $rc -eq 0 ] || tail -30 "${out%.jsonl}.err"; return $rc ;;
    *) echo "unknown job: $kind"; return 64 ;;
  esac
}

for j in "$@"; do
  echo "== $j"
  job $j || exit $?
done
