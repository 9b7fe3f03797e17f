# Round-2 re-entry baseline: full -m gpu suite, default bench (c2), c3 bench, kernel trace of c2.
set -o pipefail
T=${1:-r02g}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -q -rA --maxfail=20 --timeout 400 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline --steps 100 > gpurun_out/${T}_bench_c3.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/${T}_prof_c2.log 2>&1
