set -o pipefail
T=${1:-r02c}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python -u tools/dw_bench.py --batch 1024 > gpurun_out/${T}_dw1024.log 2>&1 && \
timeout -k 10 120 python -u tools/dw_bench.py --batch 4096 --nout 1678 > gpurun_out/${T}_dw4096.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1
