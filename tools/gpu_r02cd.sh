# Final validation: full GPU suite (scoring default batch changed), DP schedule overhead at c2 / c4 with the new defaults.
set -o pipefail
T=${1:-r02cd}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
timeout -k 10 150 python -u tools/dp_overhead.py 100 1024 ae > gpurun_out/${T}_dp.log 2>&1 && \
timeout -k 10 150 python -u tools/dp_overhead.py 100 4096 vib_ae >> gpurun_out/${T}_dp.log 2>&1
