# Tail schedule at c2/c3: dW of layers 1..dw_main-1 on the tail stream (MMAD_DW_TAIL) and the main-stream dW count (MMAD_DW_MAIN).
set -o pipefail
T=${1:-r02bo}
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
for v in "base:X=1" "tail:MMAD_DW_TAIL=1" "main3tail:MMAD_DW_MAIN=3 MMAD_DW_TAIL=1" "main1:MMAD_DW_MAIN=1" "main3:MMAD_DW_MAIN=3"; do
  tag=${v%%:*}; e=${v#*:}
  for c in c2 c3; do
    env $e timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; exit 1; }
    tail -1 /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $c', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
  done
done
done
