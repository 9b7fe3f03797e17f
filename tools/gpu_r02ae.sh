set -o pipefail
T=${1:-r02ae}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-probe --steps 200 --warmup 20 --config c3"
run() { name=$1; shift; env "$@" timeout -k 10 150 $B > gpurun_out/${T}_${name}.log 2>&1; }
run base1 && run sk0_1 MMAD_SPLITK_DW_BLOCKS=1 && run both_1 MMAD_SPLITK_DW_BLOCKS=1 MMAD_DW_SPLIT=0 && run split0_1 MMAD_DW_SPLIT=0 && \
run base2 && run sk0_2 MMAD_SPLITK_DW_BLOCKS=1 && run both_2 MMAD_SPLITK_DW_BLOCKS=1 MMAD_DW_SPLIT=0 && run split0_2 MMAD_DW_SPLIT=0 && \
run sk256 MMAD_SPLITK_DW_BLOCKS=256 && run sk128 MMAD_SPLITK_DW_BLOCKS=128
