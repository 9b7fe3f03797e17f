# Schedule-equivalence tests.
set -o pipefail
T=${1:-r02bz}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_schedules.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
