#!/bin/bash
# The one GPU-box launcher (replaces the per-round one-off scripts).  Every step runs under its own
# time limit, steps are chained with &&, and everything lands in gpurun_out/TAG.
#
#   bash tools/gpu.sh TAG tests [PYTEST_ARGS...]   pytest -m gpu over tests/ (or the given args)
#   bash tools/gpu.sh TAG bench [BENCH_ARGS...]    one bench.py line (default: the headline, no CPU leg)
#   bash tools/gpu.sh TAG configs                  bench lines of configs 2 / 4 / 5 (no CPU leg)
#   bash tools/gpu.sh TAG train [ARGS...]          tools/bench_train.py --profile
#   bash tools/gpu.sh TAG trace                    rocprofv3 --kernel-trace --stats of the bench command
#   bash tools/gpu.sh TAG pmc [HEAD]               FETCH_SIZE and WRITE_SIZE passes (separate runs) -> pmc_traffic.json
#   bash tools/gpu.sh TAG sq [SCRIPT [ARGS...]]    SQ stall / mix / LDS / MFMA-busy passes -> summary.txt, mfma_util.txt
#                                                  (CATSEG_HIP_LIB=... in the environment: another library, for A/B)
#   bash tools/gpu.sh TAG final [HEAD]             tests + smoke + headline (with CPU leg) + configs + trace + pmc + sq
#   bash tools/gpu.sh TAG final1                    the first half of final: tests + smoke + headline + configs
#   bash tools/gpu.sh TAG final2 [HEAD]             the second half: trace + pmc + sq + the training step
#   bash tools/gpu.sh TAG micro SCRIPT [ARGS...]   one tools/micro_*.py run
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=${1:?usage: gpu.sh TAG CMD [ARGS]}
CMD=${2:?usage: gpu.sh TAG CMD [ARGS]}
shift 2
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1

tests() {
  if [ $# -eq 0 ]; then set -- tests -m gpu; fi
  timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1
}
bench() {
  if [ $# -eq 0 ]; then set -- --cpu-images 0; fi
  timeout -k 10 400 python -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"
}
configs() {
  timeout -k 10 300 python -u bench.py --config 2 --cpu-images 0 > "$O/bench_config2.json" 2>> "$O/bench.err" &&
  timeout -k 10 300 python -u bench.py --config 4 --cpu-images 0 > "$O/bench_config4.json" 2>> "$O/bench.err" &&
  timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 --cpu-images 0 > "$O/bench_config5.json" 2>> "$O/bench.err"
}
train() {
  timeout -k 10 600 python -u tools/bench_train.py --profile "$@" > "$O/bench_train.json" 2> "$O/bench_train.err"
}
trace() {
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-images 0 > "$O/trace.log" 2>&1)
}
pmc() {
  (cd /tmp &&
   timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$O/pmc_fetch" -o run -- \
     python3 "$R/tools/pmc_step.py" > "$O/pmc_fetch.log" 2>&1 &&
   timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$O/pmc_write" -o run -- \
     python3 "$R/tools/pmc_step.py" > "$O/pmc_write.log" 2>&1) &&
  python3 tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" -o "$O/pmc_traffic.json" --head "${1:-unknown}" \
    > "$O/pmc_traffic.txt" 2>&1
}
sq() {
  local PY=${1:-tools/pmc_step.py}
  shift || true                       # the rest: the script's arguments (e.g. micro_decoder.py's knob values)
  (cd /tmp &&
   timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
     SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$O/sqa" -o run -- python3 "$R/$PY" "$@" \
     > "$O/sqa.log" 2>&1 &&
   timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
     SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$O/sqb" -o run -- python3 "$R/$PY" "$@" \
     > "$O/sqb.log" 2>&1) &&
  python3 tools/pmc_summary.py "$O/sqa" "$O/sqb" --top 30 > "$O/summary.txt" 2>&1 &&
  python3 tools/mfma_util.py "$O/sqb" --top 40 > "$O/mfma_util.txt" 2>&1
}
smoke() {
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
}
micro() {
  local S=${1:?micro SCRIPT}
  shift
  timeout -k 10 400 python -u "tools/$S" "$@" > "$O/${S%.py}.log" 2>&1
}

case "$CMD" in
  tests) tests "$@" ;;
  bench) bench "$@" ;;
  configs) configs ;;
  train) train "$@" ;;
  trace) trace ;;
  pmc) pmc "$@" ;;
  sq) sq "$@" ;;
  micro) micro "$@" ;;
  smoke) smoke ;;
  final) tests && smoke && bench && configs && trace && pmc "$@" && sq ;;
  final1) tests && smoke && bench --cpu-images -1 && configs ;;
  final2) trace && pmc "$@" && sq && train ;;
  *) echo "unknown command $CMD" >&2; exit 2 ;;
esac
