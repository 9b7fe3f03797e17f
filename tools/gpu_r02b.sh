# e2e/VIB/metrics diagnostics with prints, then kernel traces of c2 and c3.
set -o pipefail
T=${1:-r02b}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s -q -rA --timeout 300 --timeout-method thread tests/test_gpu_e2e.py tests/test_gpu_vib_full.py "tests/test_gpu_gemm.py::test_splitk_timeout_is_reported_not_combined" > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/${T}_prof_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c3 -o run -- python3 bench.py --config c3 --no-cpu-baseline --steps 30 --warmup 10 > gpurun_out/${T}_prof_c3.log 2>&1
