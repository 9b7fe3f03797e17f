# dW(+Adam) microbenchmark per tile and host-side per-call costs
set -o pipefail
T=${1:-r02h}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 60 ./tools/ubench_host > gpurun_out/${T}_ubench_host.log 2>&1 && \
timeout -k 10 120 python -u tools/dw_bench.py --batch 1024 > gpurun_out/${T}_dw1024.log 2>&1 && \
timeout -k 10 120 python -u tools/dw_bench.py --batch 1024 --nout 1268 --nin 1658 > gpurun_out/${T}_dw1024_l2.log 2>&1 && \
timeout -k 10 120 python -u tools/dw_bench.py --batch 4096 --nout 1678 > gpurun_out/${T}_dw4096.log 2>&1
