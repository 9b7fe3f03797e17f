# Data-parallel schedule cost on one GPU (loopback exchange) at c2 and c4 sizes, and its timeline at c4.
set -o pipefail
T=${1:-r02bi}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 150 python -u tools/dp_overhead.py 100 1024 ae > gpurun_out/${T}_dp.log 2>&1 && \
timeout -k 10 150 python -u tools/dp_overhead.py 100 4096 vib_ae >> gpurun_out/${T}_dp.log 2>&1
