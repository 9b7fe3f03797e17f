# BN kernel launch shapes at c3: bn_bwd_apply_k partial loads per round trip (PU), bn_fold_k rows per block (RPT); full GPU suite first.
set -o pipefail
T=${1:-r02bj}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config c3"
for rep in 1 2; do
for v in "pu8_rpt2:MMAD_BNB_PU=8" "pu16_rpt2:X=1" "pu16_rpt4:MMAD_FOLD_RPT=4"; do
  tag=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 150 $B > gpurun_out/${T}_${tag}.log 2>&1 || exit 1
  tail -1 gpurun_out/${T}_${tag}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
done
done
