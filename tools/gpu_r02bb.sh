# Step breakdown (host vs GPU per phase) at c2 and c3, knob variants, and a host-side HIP trace.
set -o pipefail
T=${1:-r02bb}
mkdir -p gpurun_out && export TMPDIR=/tmp
S="python -u tools/step_breakdown.py --steps 200"
timeout -k 10 120 $S --tag c2 > gpurun_out/${T}_brk.log 2>&1 && \
MMAD_DW_MAIN=10 timeout -k 10 120 $S --tag c2_serial >> gpurun_out/${T}_brk.log 2>&1 && \
MMAD_BN_MODE=1 timeout -k 10 120 $S --tag c2_fold >> gpurun_out/${T}_brk.log 2>&1 && \
timeout -k 10 120 $S --tag c3 --batch 4096 --model vib_ae >> gpurun_out/${T}_brk.log 2>&1 && \
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace -d /tmp/ht -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 30 --warmup 10 > gpurun_out/${T}_ht.log 2>&1 && \
python3 tools/host_gaps.py /tmp/ht > gpurun_out/${T}_host_gaps.txt 2>&1
