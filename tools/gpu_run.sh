# One parameterised GPU-box runner (replaces the per-call one-shot scripts).
# Usage on the box:  bash tools/gpu_run.sh <tag> <step> [<step> ...]
# Steps (run in order; the first failure ends the call, no GPU step after it):
#   tests            full `pytest -m gpu` suite
#   tests:<expr>     `pytest -m gpu -k <expr>` ('+' -> ' ', e.g. tests:bn_fused+or+dp)
#   smoke            __graft_entry__.smoke()
#   bench[:<args>]   python bench.py <args, commas -> spaces>
#   prof[:<args>]    rocprofv3 --kernel-trace --stats of bench.py <args>
#   py:<script,args> python <script> <args>          (tools/*.py helpers)
#   bin:<path,args>  a prebuilt binary (tools/ubench_*)
#   trace:<script,args>  rocprofv3 --kernel-trace --stats of python <script> <args>
#   htrace:<script,args> rocprofv3 --hip-trace --kernel-trace (host API timeline)
#   pmc:<ctr+ctr>:<script,args>  one rocprofv3 --pmc pass (counters joined by '+')
# Every GPU step runs under its own timeout; logs go to gpurun_out/<tag>_*.
set -o pipefail
T=${1:?tag}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
# heartbeat: a fresh box's first `import torch` can take minutes with nothing
# printed; every step still runs under its own time limit
( while sleep 30; do date +%s >> gpurun_out/${T}_heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  log=gpurun_out/${T}_${i}_${kind}.log
  case "$kind" in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -k "${arg//+/ }" --timeout 300 --timeout-method thread > "$log" 2>&1
      else
        timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > "$log" 2>&1
      fi ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 ;;
    bench)
      timeout -k 10 400 python -u bench.py ${arg//,/ } > "$log" 2>&1 ;;
    prof)
      # keep the --stats CSVs and a per-grid summary; the trace database stays on the box.
      # c5 replays one captured hipGraph per pass: rocprofiler-sdk's kernel-trace
      # intercept faults on HIP's batched graph packets after some hundred replays
      # (profiles/r10/r10a_c5_rocprof_segv/ANALYSIS.txt), so those graphs dispatch
      # kernel by kernel under the profiler
      pc=1; [[ "$arg" == *c5* ]] && pc=0
      DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${T}_${i}_prof -o run -- \
        python3 bench.py ${arg//,/ } > "$log" 2>&1 &&
        mkdir -p gpurun_out/${T}_${i}_prof &&
        { find /tmp/${T}_${i}_prof -name "*stats*.csv" -exec cp {} gpurun_out/${T}_${i}_prof/ \; ; true; } &&
        python3 tools/prof_db.py "$(find /tmp/${T}_${i}_prof -name '*.db' | head -1)" \
          > gpurun_out/${T}_${i}_prof/kstats.txt 2>&1 &&
        python3 tools/prof_db.py "$(find /tmp/${T}_${i}_prof -name '*.db' | head -1)" --by-grid \
          > gpurun_out/${T}_${i}_prof/kstats_bygrid.txt 2>&1 &&
        python3 tools/prof_step.py "$(find /tmp/${T}_${i}_prof -name '*.db' | head -1)" --last 20 \
          > gpurun_out/${T}_${i}_prof/timeline.txt 2>&1
      rc_=$?; rm -rf /tmp/${T}_${i}_prof; (exit $rc_) ;;
    py)
      timeout -k 10 400 python -u ${arg//,/ } > "$log" 2>&1 ;;
    bin)
      timeout -k 10 300 ${arg//,/ } > "$log" 2>&1 ;;
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_${i}_trace -o run -- \
        python3 ${arg//,/ } > "$log" 2>&1 ;;
    htrace)
      # summarised on the box (the raw trace is large), then removed
      timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace -d /tmp/${T}_${i}_htrace -o run -- \
        python3 ${arg//,/ } > "$log" 2>&1 &&
        python3 tools/hip_api_stats.py /tmp/${T}_${i}_htrace --steps 20 > gpurun_out/${T}_${i}_api.txt 2>&1 &&
        python3 tools/host_gaps.py /tmp/${T}_${i}_htrace > gpurun_out/${T}_${i}_gaps.txt 2>&1 &&
        python3 tools/prof_step.py "$(ls /tmp/${T}_${i}_htrace/*/*.db /tmp/${T}_${i}_htrace/*.db 2>/dev/null | head -1)" \
          --last 15 > gpurun_out/${T}_${i}_timeline.txt 2>&1
      rc_=$?; rm -rf /tmp/${T}_${i}_htrace; (exit $rc_) ;;
    pmc)
      ctr=${arg%%:*}
      cmd=${arg#*:}
      timeout -s KILL 120 rocprofv3 --pmc ${ctr//+/ } -d gpurun_out/${T}_${i}_pmc -o run -- \
        python3 ${cmd//,/ } > "$log" 2>&1 ;;
    *)
      echo "unknown step $step" >&2; exit 2 ;;
  esac
  rc=$?
  echo "[gpu_run] step $i ($step) exit $rc"
  if [ $rc -ne 0 ]; then
    tail -30 "$log"
    exit $rc
  fi
done
