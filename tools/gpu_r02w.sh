set -o pipefail
T=${1:-r02w}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --steps 100 --warmup 20"
timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3.log 2>&1 && \
MMAD_GEMM_TILE_ADAM=3 timeout -k 10 150 $B --config c3 --no-probe > gpurun_out/${T}_c3_t3.log 2>&1 && \
timeout -k 10 100 $B > gpurun_out/${T}_c2.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
