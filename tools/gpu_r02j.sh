# dW split-K sweep (B=1024 AE, B=4096 VIB-AE), schedule knobs on the c2/c3 bench, split-K/parity tests
set -o pipefail
T=${1:-r02j}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-probe --steps 100 --warmup 20"
timeout -k 10 200 python -u tools/splitk_dw_sweep.py 1024 > gpurun_out/${T}_splitk_dw1024.log 2>&1 && \
timeout -k 10 300 python -u tools/splitk_dw_sweep.py 4096 1 > gpurun_out/${T}_splitk_dw4096.log 2>&1 && \
timeout -k 10 100 $B > gpurun_out/${T}_c2_default.log 2>&1 && \
MMAD_GEMM_SPLITK_DW=1 timeout -k 10 100 $B > gpurun_out/${T}_c2_nosplit.log 2>&1 && \
MMAD_DW_TAIL=1 timeout -k 10 100 $B > gpurun_out/${T}_c2_tail.log 2>&1 && \
MMAD_SIDE_CUS=128 timeout -k 10 100 $B > gpurun_out/${T}_c2_cus128.log 2>&1 && \
MMAD_SIDE_CUS=64 timeout -k 10 100 $B > gpurun_out/${T}_c2_cus64.log 2>&1 && \
MMAD_SIDE_CUS=192 timeout -k 10 100 $B > gpurun_out/${T}_c2_cus192.log 2>&1 && \
timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3_default.log 2>&1 && \
MMAD_GEMM_SPLITK_DW=1 timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3_nosplit.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -q -rA --timeout 300 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_parity.py tests/test_gpu_vib_full.py > gpurun_out/${T}_pytest.log 2>&1
