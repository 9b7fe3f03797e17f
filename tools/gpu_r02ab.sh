set -o pipefail
T=${1:-r02ab}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python tools/gemm_phase.py 4096 0,1,8 0,2,5,3 bwd_w,bwd_data > gpurun_out/${T}_phase_dw.log 2>&1 && \
B="python -u bench.py --no-cpu-baseline --steps 100 --warmup 20 --config c3"
timeout -k 10 150 $B > gpurun_out/${T}_c3.log 2>&1 && \
MMAD_GEMM_TILE_ADAM=2 timeout -k 10 150 $B > gpurun_out/${T}_c3_t2.log 2>&1
