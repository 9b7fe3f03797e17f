set -o pipefail
T=${1:-r02r}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u tools/gemm_phase.py 1024 0,3,4,8 > gpurun_out/${T}_gemm_phase.log 2>&1 && \
timeout -k 10 60 ./tools/ubench_host > gpurun_out/${T}_ubench_host.log 2>&1
