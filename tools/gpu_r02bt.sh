# A/B: loss reduction on the side stream (MMAD_LOSS_SIDE=1, default) vs at the end of the main stream.
set -o pipefail
T=${1:-r02bt}
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2 3; do for ls in 1 0; do for c in c2 c3; do
  MMAD_LOSS_SIDE=$ls timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 400 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; exit 1; }
  grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('side=$ls $c', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
done; done; done
