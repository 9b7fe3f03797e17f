# Tile of the Adam-fused dW GEMMs on the main-stream tail (knob 8) after the LDS-DMA fix, c2 and c3.
set -o pipefail
T=${1:-r02bk}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --steps 300"
for c in c2 c3; do
for t in -1 0 1 3 4 5; do
  MMAD_GEMM_TILE_ADAM_MAIN=$t timeout -k 10 150 $B --config $c > gpurun_out/${T}_${c}_t${t}.log 2>&1 || exit 1
  tail -1 gpurun_out/${T}_${c}_t${t}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c tile_main=$t', d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['frac'])" >> gpurun_out/${T}_sum.txt
done
done
