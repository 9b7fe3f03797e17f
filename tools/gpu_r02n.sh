# new defaults (bf16: fused BN up to 2048 rows, fold above): whole gpu suite, default bench (c2, full line), c3 bench
set -o pipefail
T=${1:-r02n}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline --steps 100 > gpurun_out/${T}_bench_c3.log 2>&1
