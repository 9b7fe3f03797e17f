# Second schedule sweep on the new defaults (c2: main-stream dW count, tail stream, Adam tile, BN mode; c3: split tail, Adam tile, BN mode).
set -o pipefail
T=${1:-r02bx}
mkdir -p gpurun_out && export TMPDIR=/tmp
run() { # tag config env...
  local tag=$1 c=$2; shift 2
  env "$@" timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; return 1; }
  grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $c', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
}
for rep in 1 2; do
  run base c2 X=1 && run main1 c2 MMAD_DW_MAIN=1 && run main3 c2 MMAD_DW_MAIN=3 && run tail c2 MMAD_DW_TAIL=1 && \
  run adam4 c2 MMAD_GEMM_TILE_ADAM=4 && run adam5 c2 MMAD_GEMM_TILE_ADAM=5 && run fold c2 MMAD_BN_MODE=1 && \
  run base c3 X=1 && run split c3 MMAD_DW_SPLIT=1 && run adam3 c3 MMAD_GEMM_TILE_ADAM=3 && run adam0 c3 MMAD_GEMM_TILE_ADAM=0 && \
  run fused c3 MMAD_BN_FUSED_MAX_ROWS=4096 && run prio c3 MMAD_SIDE_PRIO=1 || exit 1
done
