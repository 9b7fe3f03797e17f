set -o pipefail
T=${1:-r02y}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_e2e.py -m gpu -q -rA -k "nap or e2e or auroc" --timeout 200 --timeout-method thread > gpurun_out/${T}_nap.log 2>&1
