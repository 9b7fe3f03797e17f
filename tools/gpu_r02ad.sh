# schedule / tile re-sweep after the asm LDS-DMA change
set -o pipefail
T=${1:-r02ad}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-probe --steps 100 --warmup 20"
run() { name=$1; shift; env "$@" timeout -k 10 150 $B $CFG > gpurun_out/${T}_${name}.log 2>&1; }
CFG=""
run c2_base && run c2_ta0 MMAD_GEMM_TILE_ADAM=0 && run c2_ta5 MMAD_GEMM_TILE_ADAM=5 && \
run c2_split1 MMAD_DW_SPLIT=1 && run c2_main1 MMAD_DW_MAIN=1 && run c2_main0 MMAD_DW_MAIN=0 && \
CFG="--config c3" && \
run c3_base && run c3_ta3 MMAD_GEMM_TILE_ADAM=3 && run c3_ta5 MMAD_GEMM_TILE_ADAM=5 && \
run c3_bn2 MMAD_BN_MODE=2 MMAD_BN_FUSED_MAX_ROWS=4096 && run c3_split0 MMAD_DW_SPLIT=0 && \
run c3_sk0 MMAD_SPLITK_DW_BLOCKS=1
