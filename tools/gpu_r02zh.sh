# Native all-reduce self-test + DP tests, then the N=2 harness on one GPU.
set -o pipefail
T=${1:-r02zh}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -m gpu -q -rf --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
MMAD_BENCH_SHARED_GPU=1 timeout -k 10 150 python -u bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_n2.log 2>&1
