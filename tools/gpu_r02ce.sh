# Forced forward / bwd-data tiles in the step (knobs 7 / 6) vs the per-shape autotune, c2 and c3.
set -o pipefail
T=${1:-r02ce}
mkdir -p gpurun_out && export TMPDIR=/tmp
run() { local tag=$1 c=$2; shift 2
  env "$@" timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; return 1; }
  grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $c', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt; }
for c in c2 c3; do
  run auto $c X=1 || exit 1
  for t in 0 1 3 4 5; do run fwd$t $c MMAD_GEMM_TILE_FWD=$t || exit 1; run bd$t $c MMAD_GEMM_TILE_BWD_DATA=$t || exit 1; done
  run auto $c X=1 || exit 1
done
