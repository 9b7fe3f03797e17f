set -o pipefail
T=${1:-r02af}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 30 --warmup 10 > gpurun_out/${T}_prof_c2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c3 -o run -- python3 bench.py --config c3 --no-cpu-baseline --no-probe --steps 30 --warmup 10 > gpurun_out/${T}_prof_c3.log 2>&1
