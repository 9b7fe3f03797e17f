# XCD tile-group height override (MMAD_GEMM_GROUP_M) at c2 / c3 vs the per-shape rule.
set -o pipefail
T=${1:-r02ca}
mkdir -p gpurun_out && export TMPDIR=/tmp
for c in c2 c3; do for g in -1 1 2 4 8 16; do
  MMAD_GEMM_GROUP_M=$g timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; exit 1; }
  grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gm=$g $c', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
done; done
