# Backward BN schedule override at c3 (fold forward + fused backward) and c2, with an equivalence check of losses vs the default.
set -o pipefail
T=${1:-r02cg}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn_fused.py -m gpu -q -rf --timeout 200 --timeout-method thread -k fold_forward > gpurun_out/${T}_pytest.log 2>&1 || exit 1
for rep in 1 2; do for v in "base:X=1" "fbwd:MMAD_BN_MODE_BWD=2"; do for c in c3 c2; do
  tag=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; exit 1; }
  grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $c', d['ms_per_step'], d['final_loss'])" >> gpurun_out/${T}_sum.txt
done; done; done
