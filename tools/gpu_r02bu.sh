# Schedule knobs re-swept on the current code: ping-pong weight shadows, event coalescing, side-stream priority, main-stream dW count with shadows.
set -o pipefail
T=${1:-r02bu}
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
for v in "base:X=1" "pair:MMAD_SHADOW_PAIR=1" "pair_main1:MMAD_SHADOW_PAIR=1 MMAD_DW_MAIN=1" "ev2:MMAD_EV_EVERY=2" "prio:MMAD_SIDE_PRIO=1"; do
  tag=${v%%:*}; e=${v#*:}
  for c in c2 c3; do
    env $e timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; exit 1; }
    grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $c', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
  done
done
done
