# Timeline of the data-parallel schedule on one GPU (loopback exchange) at c4's 4096 windows per GPU.
set -o pipefail
T=${1:-r02cj}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/dp -o run -- python3 tools/dp_overhead.py 40 4096 vib_ae > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/prof_step.py $(find /tmp/dp -name "*.db" | head -1) --last 10 > gpurun_out/${T}_timeline.txt 2>&1
