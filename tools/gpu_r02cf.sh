# A/B at c2: autotuned forward / bwd-data tiles vs 64x64 forced for both.
set -o pipefail
T=${1:-r02cf}
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2 3; do for v in "auto:X=1" "t3:MMAD_GEMM_TILE_FWD=3 MMAD_GEMM_TILE_BWD_DATA=3"; do
  tag=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 400 > /tmp/b.txt 2>&1 || exit 1
  grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag c2', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
done; done
