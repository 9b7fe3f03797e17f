# A/B: where the DP small bucket joins the comm stream (after bwd-data of layer 1 vs at layer 0), c2 / c4 sizes, loopback exchange.
set -o pipefail
T=${1:-r02cn}
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2 3; do for at in 1 0; do
  MMAD_DP_SMALL_AT=$at timeout -k 10 150 python -u tools/dp_overhead.py 100 1024 ae 2>&1 | grep fused | sed "s/^/at=$at /" >> gpurun_out/${T}_sum.txt || exit 1
  MMAD_DP_SMALL_AT=$at timeout -k 10 150 python -u tools/dp_overhead.py 100 4096 vib_ae 2>&1 | grep fused | sed "s/^/at=$at /" >> gpurun_out/${T}_sum.txt || exit 1
done; done
