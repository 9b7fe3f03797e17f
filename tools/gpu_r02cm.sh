# Small DP bucket queued ahead of layers 1 and 0 on the comm stream: DP tests (loopback bit-exactness), DP overhead at c2/c4, DP timeline.
set -o pipefail
T=${1:-r02cm}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
timeout -k 10 150 python -u tools/dp_overhead.py 100 1024 ae > gpurun_out/${T}_dp.log 2>&1 && \
timeout -k 10 150 python -u tools/dp_overhead.py 100 4096 vib_ae >> gpurun_out/${T}_dp.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/dp -o run -- python3 tools/dp_overhead.py 40 4096 vib_ae > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/prof_step.py $(find /tmp/dp -name "*.db" | head -1) --last 10 > gpurun_out/${T}_timeline.txt 2>&1
