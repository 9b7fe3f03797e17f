# library GEMM calibration at B=1024 and 4096
set -o pipefail
T=${1:-r02i}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u tools/blas_cmp.py 1024 > gpurun_out/${T}_blas1024.log 2>&1 && \
timeout -k 10 200 python -u tools/blas_cmp.py 4096 > gpurun_out/${T}_blas4096.log 2>&1
