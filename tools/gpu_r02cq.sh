# c2 with the ping-pong schedule under the current defaults (event coalescing 2): 1 / 2 / 3 main-stream dW GEMMs vs single shadow.
set -o pipefail
T=${1:-r02cq}
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do for v in "base:X=1" "ping_m2:MMAD_SHADOW_PAIR_ROWS=0 MMAD_DW_MAIN_PING=2" "ping_m1:MMAD_SHADOW_PAIR_ROWS=0 MMAD_DW_MAIN_PING=1" "ping_m3:MMAD_SHADOW_PAIR_ROWS=0 MMAD_DW_MAIN_PING=3"; do
  tag=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 > /tmp/b.txt 2>&1 || exit 1
  grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag c2', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
done; done
