# Data-parallel NoveltyDetecter (2 ranks on one GPU over gloo) + DP tests.
set -o pipefail
T=${1:-r02bl}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_e2e.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
