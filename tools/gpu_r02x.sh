set -o pipefail
T=${1:-r02x}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_layers.py -m gpu -q -rA -k activation --timeout 120 --timeout-method thread > gpurun_out/${T}_act.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
