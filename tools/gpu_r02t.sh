# warp-specialised dW+Adam kernel: bit-identity tests, standalone cold timing (ws on/off), benches
set -o pipefail
T=${1:-r02t}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -rA --timeout 120 --timeout-method thread tests/test_gpu_dw_ws.py > gpurun_out/${T}_pytest_ws.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_pytest_ws.log; if [ $rc -ne 0 ]; then exit $rc; fi
D="python3 tools/dw_one.py 1024 1658 2048 40 3"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_ws -o run -- $D > gpurun_out/${T}_prof_ws.log 2>&1 && \
MMAD_DW_WS=0 timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_nows -o run -- $D > gpurun_out/${T}_prof_nows.log 2>&1 && \
MMAD_DW_WS_BLOCKS=128 timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_ws128 -o run -- $D > gpurun_out/${T}_prof_ws128.log 2>&1 && \
timeout -k 10 150 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_c2.log 2>&1 && \
MMAD_DW_WS=0 timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe > gpurun_out/${T}_c2_nows.log 2>&1 && \
MMAD_DW_WS_BLOCKS=128 timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe > gpurun_out/${T}_c2_ws128.log 2>&1 && \
timeout -k 10 150 python -u bench.py --config c3 --no-cpu-baseline --steps 100 > gpurun_out/${T}_c3.log 2>&1 && \
MMAD_DW_WS=0 timeout -k 10 150 python -u bench.py --config c3 --no-cpu-baseline --no-probe --steps 100 > gpurun_out/${T}_c3_nows.log 2>&1
