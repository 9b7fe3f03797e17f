set -o pipefail
T=${1:-r02f}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 60 ./tools/ubench_host > gpurun_out/${T}_ubench_host.log 2>&1 && \
timeout -k 10 120 python -u tools/dw_bench.py > gpurun_out/${T}_dw.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -q -s -rA --timeout 300 --timeout-method thread tests/test_gpu_vib_full.py tests/test_gpu_layers.py > gpurun_out/${T}_pytest.log 2>&1
