# r01r: GPU tests + smoke + default bench line + kernel trace, then the
# main-stream Adam-dW tile sweep (knob 8) at DW_MAIN 2 and 3.
set -o pipefail
T=r01r
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 200 python -u tools/tile_adam_sweep.py 8 > gpurun_out/${T}_sweep8.log 2>&1 && \
MMAD_DW_MAIN=3 timeout -k 10 200 python -u tools/tile_adam_sweep.py 8 > gpurun_out/${T}_sweep8_dw3.log 2>&1 && \
MMAD_DW_MAIN=1 timeout -k 10 200 python -u tools/tile_adam_sweep.py 8 > gpurun_out/${T}_sweep8_dw1.log 2>&1
