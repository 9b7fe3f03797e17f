# Schedule knob combinations: c2 (event coalescing, side priority) and c3 (ping-pong shadows with 0/1 main-stream dW, + coalescing / priority).
set -o pipefail
T=${1:-r02bv}
mkdir -p gpurun_out && export TMPDIR=/tmp
run() { # tag config env...
  local tag=$1 c=$2; shift 2
  env "$@" timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; return 1; }
  grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $c', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
}
for rep in 1 2; do
  run base c2 X=1 && run ev2 c2 MMAD_EV_EVERY=2 && run ev3 c2 MMAD_EV_EVERY=3 && run ev2prio c2 MMAD_EV_EVERY=2 MMAD_SIDE_PRIO=1 && \
  run ev4 c2 MMAD_EV_EVERY=4 && \
  run base c3 X=1 && run p_m1 c3 MMAD_SHADOW_PAIR=1 MMAD_DW_MAIN=1 && run p_m0 c3 MMAD_SHADOW_PAIR=1 MMAD_DW_MAIN=0 && \
  run p_m1_ev2 c3 MMAD_SHADOW_PAIR=1 MMAD_DW_MAIN=1 MMAD_EV_EVERY=2 && run p_m1_prio c3 MMAD_SHADOW_PAIR=1 MMAD_DW_MAIN=1 MMAD_SIDE_PRIO=1 && \
  run p_m2_ev2 c3 MMAD_SHADOW_PAIR=1 MMAD_EV_EVERY=2 || exit 1
done
