# Non-temporal Adam-state accesses (knob 15) vs default, c2 and c3 bench lines.
set -o pipefail
T=${1:-r02bc}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --steps 300"
for nt in 0 1 0 1; do
  MMAD_ADAM_NT=$nt timeout -k 10 150 $B > gpurun_out/${T}_c2_nt${nt}.log 2>&1 || exit 1
  tail -1 gpurun_out/${T}_c2_nt${nt}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 nt=$nt', d['ms_per_step'], d['roofline']['avg_us'])" >> gpurun_out/${T}_sum.txt
  MMAD_ADAM_NT=$nt timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3_nt${nt}.log 2>&1 || exit 1
  tail -1 gpurun_out/${T}_c3_nt${nt}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 nt=$nt', d['ms_per_step'], d['roofline']['avg_us'])" >> gpurun_out/${T}_sum.txt
done
