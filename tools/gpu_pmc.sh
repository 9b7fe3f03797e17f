# PMC passes of the roofline GEMMs (one counter group per rocprofv3 run, each
# under its own time limit; no --pmc beside a trace domain) + one kernel-trace
# pass, summarised by tools/pmc_gemm.py into profiles/<tag>_<w>_pmc_<kind>.json
# (copied to gpurun_out/).  The summaries carry the GEMM sources' hash, which
# bench.py checks before it reports their traffic.
# Usage: bash tools/gpu_pmc.sh <tag> [workloads: c3e c2e c3w c2w c5s]
set -o pipefail
T=$1; shift
WL=${*:-c3e c3w c2e c2w}
mkdir -p gpurun_out && export TMPDIR=/tmp
pass() {   # pass <dir> <counters|trace> <cmd...>
  local d=$1 c=$2; shift 2
  if [ "$c" = trace ]; then
    timeout -k 10 90 rocprofv3 --kernel-trace -d gpurun_out/$d -o run -- "$@" > gpurun_out/$d.log 2>&1
  else
    timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/$d -o run -- "$@" > gpurun_out/$d.log 2>&1
  fi
  local rc=$?; echo "[pmc] $d ($c) exit $rc"; return $rc
}
for w in $WL; do
  case $w in
    c3e) kind=traffic; B=4096; M=vib_ae; CMD="python3 tools/gemm_one.py fwd 0 4096 40 -1 -1 vib_ae";;
    c2e) kind=traffic; B=1024; M=ae;     CMD="python3 tools/gemm_one.py fwd 0 1024 40 -1 -1 ae";;
    c3w) kind=dw;      B=4096; M=vib_ae; CMD="python3 tools/dw_one.py 4096 1678 2048 40 -2";;
    c2w) kind=dw;      B=1024; M=ae;     CMD="python3 tools/dw_one.py 1024 1658 2048 40 -2";;
    c5s) kind=score;   B=65536; M=ae;    CMD="python3 tools/score_one.py 65536 20";;
    *) echo "unknown workload $w"; exit 2;;
  esac
  for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "hit TCC_HIT_sum TCC_MISS_sum" \
           "mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    set -- $p; n=$1; shift
    pass ${T}_${w}_pmc_$n "$*" $CMD || exit 1
  done
  pass ${T}_${w}_trace trace $CMD || exit 1
  python3 tools/pmc_gemm.py $kind ${T}_${w} $B $M > gpurun_out/${T}_${w}_summary.json || exit 1
  cp profiles/${T}_${w}_pmc_${kind}.json gpurun_out/ || exit 1
  # the per-pass databases are tens of MB each (gpurun copies back <= 64 MiB)
  rm -rf gpurun_out/${T}_${w}_pmc_*/ gpurun_out/${T}_${w}_trace/
done
ls gpurun_out/${T}_*
