# BN schedule per direction: fused forward + apply-kernel backward (MMAD_BN_FUSED_MAX_ROWS=4096 MMAD_BN_MODE_BWD=0) vs the defaults, c3 and c2.
set -o pipefail
T=${1:-r02ci}
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do for v in "base:X=1" "ffwd_abwd:MMAD_BN_FUSED_MAX_ROWS=4096 MMAD_BN_MODE_BWD=0"; do for c in c3 c2; do
  tag=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; exit 1; }
  grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $c', d['ms_per_step'], d['final_loss'])" >> gpurun_out/${T}_sum.txt
done; done; done
