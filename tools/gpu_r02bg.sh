# c3 BatchNorm schedule re-sweep after the LDS-DMA fix: fold (default above 2048 rows) vs fused vs apply.
set -o pipefail
T=${1:-r02bg}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config c3"
for rep in 1 2; do
for v in "fold" "fused:MMAD_BN_FUSED_MAX_ROWS=4096" "apply:MMAD_BN_MODE=0"; do
  tag=${v%%:*}; e=${v#*:}; [ "$e" = "$v" ] && e="X=1"
  env $e timeout -k 10 150 $B > gpurun_out/${T}_${tag}.log 2>&1 || exit 1
  tail -1 gpurun_out/${T}_${tag}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
done
done
