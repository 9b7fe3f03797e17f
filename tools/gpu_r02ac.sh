# asm LDS-DMA (no compiler vmcnt(0) before transposed fragment reads) + Adam-state prefetch
set -o pipefail
T=${1:-r02ac}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 200 python tools/gemm_phase.py 4096 0,8 0,3 bwd_w,bwd_data,fwd > gpurun_out/${T}_phase4096.log 2>&1 && \
timeout -k 10 200 python tools/gemm_phase.py 1024 0,3 3,0 bwd_w,bwd_data,fwd > gpurun_out/${T}_phase1024.log 2>&1 && \
B="python -u bench.py --no-cpu-baseline --steps 100 --warmup 20"
timeout -k 10 150 $B > gpurun_out/${T}_c2.log 2>&1 && \
MMAD_ADAM_PREFETCH=0 timeout -k 10 150 $B > gpurun_out/${T}_c2_noapf.log 2>&1 && \
timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3.log 2>&1
