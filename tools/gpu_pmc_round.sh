# Round PMC passes (one counter group per rocprofv3 run, each under its own
# time limit) for the two roofline kernels bench.py reports, at c2 and c3:
#   encoder-layer-1 forward GEMM (tools/gemm_one.py) -> gpurun_out/<tag>_{c2,c3}e_pmc_{fetch,write,hit}
#   Adam-fused dW GEMM (tools/dw_one.py)             -> gpurun_out/<tag>_{c2,c3}w_pmc_{fetch,write,hit,mfma}
# summarised at the end (below): python tools/pmc_traffic.py <tag>_c2e 1024 ae ; python tools/pmc_traffic.py <tag>_c3e 4096 vib_ae
#       python tools/pmc_dw.py <tag>_c2w 1024 1658 2048 0 ae <tile> ; ... <tag>_c3w 4096 1678 2048 0 vib_ae <tile>
# Usage: bash tools/gpu_pmc_round.sh <tag> [c2 dW tile] [c3 dW tile]   (-2 = the production shape rule)
set -o pipefail
T=$1; W2=${2:--2}; W3=${3:--2}
lab() { case $1 in 0) echo 128x128;; 3) echo 64x64;; 5) echo 128x128-4w;; *) echo "rule$1";; esac; }
mkdir -p gpurun_out && export TMPDIR=/tmp
pass() {   # pass <dir> <counters> <cmd...>
  local d=$1 c=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/$d -o run -- "$@" > gpurun_out/$d.log 2>&1
  local rc=$?; echo "[pmc] $d ($c) exit $rc"; return $rc
}
for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "hit TCC_HIT_sum TCC_MISS_sum"; do
  set -- $p; n=$1; shift
  pass ${T}_c2e_pmc_$n "$*" python3 tools/gemm_one.py fwd 0 1024 40 || exit 1
  pass ${T}_c3e_pmc_$n "$*" python3 tools/gemm_one.py fwd 0 4096 40 -1 -1 vib_ae || exit 1
done
for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "hit TCC_HIT_sum TCC_MISS_sum" "mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  set -- $p; n=$1; shift
  pass ${T}_c2w_pmc_$n "$*" python3 tools/dw_one.py 1024 1658 2048 40 $W2 || exit 1
  pass ${T}_c3w_pmc_$n "$*" python3 tools/dw_one.py 4096 1678 2048 40 $W3 || exit 1
done
# summarise on the box (the per-pass databases are tens of MB each and gpurun
# copies back at most 64 MiB) and keep only the JSON summaries + pass logs
python3 tools/pmc_traffic.py ${T}_c2e 1024 ae &&
  python3 tools/pmc_traffic.py ${T}_c3e 4096 vib_ae &&
  python3 tools/pmc_dw.py ${T}_c2w 1024 1658 2048 0 ae $(lab $W2) &&
  python3 tools/pmc_dw.py ${T}_c3w 4096 1678 2048 0 vib_ae $(lab $W3) &&
  cp profiles/${T}_*pmc_*.json gpurun_out/
rc=$?
rm -rf gpurun_out/${T}_c2e_pmc_*/ gpurun_out/${T}_c3e_pmc_*/ gpurun_out/${T}_c2w_pmc_*/ gpurun_out/${T}_c3w_pmc_*/
ls gpurun_out/${T}_* 2>/dev/null
exit $rc
