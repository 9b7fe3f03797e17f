# side-stream LDS reservation sweep (c2 and c3)
set -o pipefail
T=${1:-r02v}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-probe --steps 100 --warmup 20"
for pad in 0 32768 65536; do
  MMAD_SIDE_LDS_PAD=$pad timeout -k 10 100 $B > gpurun_out/${T}_c2_pad$pad.log 2>&1 || exit 3
  MMAD_SIDE_LDS_PAD=$pad timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3_pad$pad.log 2>&1 || exit 3
done
for pad in 0 32768; do
  MMAD_SIDE_LDS_PAD=$pad timeout -k 10 100 $B > gpurun_out/${T}_c2b_pad$pad.log 2>&1 || exit 3
done
