# Quick GPU check: tests, bench (events with / without system fence), kernel trace.
# Usage on the box: T=<tag> bash tools/gpu_quick_round.sh
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 300 > gpurun_out/${T}_bench.log 2>&1 && \
MMAD_EVENT_SYSFENCE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 300 > gpurun_out/${T}_bench_sysfence.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --no-cpu-baseline --steps 100 > gpurun_out/${T}_prof.log 2>&1
