# Large-GEMM efficiency: per-tile timing at B=4096 / 16384 and SQ counters of the 256x128 / 128x256 tiles.
set -o pipefail
T=${1:-r02bm}
mkdir -p gpurun_out && export TMPDIR=/tmp
for B in 4096 16384; do for t in 0 1 2 5; do
  timeout -k 10 60 python -u tools/gemm_time.py fwd 0 $B $t >> gpurun_out/${T}_time.txt 2>&1 || exit 1
  timeout -k 10 60 python -u tools/gemm_time.py bwd_data 1 $B $t >> gpurun_out/${T}_time.txt 2>&1 || exit 1
done; done
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
for t in 1 2; do
  timeout -s KILL 60 rocprofv3 --pmc $C1 -d /tmp/sq$t -o run -- python3 tools/gemm_time.py fwd 0 16384 $t 20 > gpurun_out/${T}_sq$t.log 2>&1 || exit 1
  python3 tools/pmc_dump.py $(find /tmp/sq$t -name "*.db" | head -1) >> gpurun_out/${T}_sq.txt 2>&1
done
