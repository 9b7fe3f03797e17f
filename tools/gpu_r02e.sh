set -o pipefail
T=${1:-r02e}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python -u tools/host_overhead.py > gpurun_out/${T}_host.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_graph -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 30 --warmup 5 > gpurun_out/${T}_prof_graph.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -q -s -rA --timeout 400 --timeout-method thread tests/test_gpu_e2e.py tests/test_gpu_vib_full.py tests/test_gpu_layers.py "tests/test_gpu_parity.py::test_graph_step_equals_eager_step" > gpurun_out/${T}_pytest.log 2>&1
