# Kernel timeline of the c2 step with the streamed Adam tail (is the consumer concurrent with its GEMM?).
set -o pipefail
T=${1:-r02be}
mkdir -p gpurun_out && export TMPDIR=/tmp
MMAD_ADAM_STREAM=1 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/ks -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 30 --warmup 10 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/prof_step.py $(find /tmp/ks -name "*.db" | head -1) --last 20 > gpurun_out/${T}_timeline.txt 2>&1
