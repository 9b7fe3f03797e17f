# r01s: GPU tests (incl. the HSR_Net producer), producer bench + kernel trace.
set -o pipefail
T=r01s
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 200 python -u bench_producer.py > gpurun_out/${T}_producer.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_producer -o run -- python3 bench_producer.py --no-cpu-baseline > gpurun_out/${T}_prof_producer.log 2>&1
