# split tail (dW GEMM + flat Adam for layers 0-1): gpu suite, c2/c3 with and without, c2 kernel trace
set -o pipefail
T=${1:-r02o}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --steps 100 --warmup 20"
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 100 $B > gpurun_out/${T}_c2_split.log 2>&1 && \
MMAD_DW_SPLIT=0 timeout -k 10 100 $B > gpurun_out/${T}_c2_fused.log 2>&1 && \
timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3_split.log 2>&1 && \
MMAD_DW_SPLIT=0 timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3_fused.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 50 --warmup 10 > gpurun_out/${T}_prof_c2.log 2>&1
