# End-of-round PMC passes (separate runs) of the Adam-fused dW GEMM that bench.py reports: c2 layer 0 (64x64) and c3 layer 0 (128x128).
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
pmc() { # tag dw_one-args
  local T=$1; shift
  local D="python3 tools/dw_one.py $*"
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_pmc_fetch -o run -- $D > gpurun_out/${T}_pmc1.log 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_pmc_write -o run -- $D > gpurun_out/${T}_pmc2.log 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${T}_pmc_hit -o run -- $D > gpurun_out/${T}_pmc3.log 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${T}_pmc_mfma -o run -- $D > gpurun_out/${T}_pmc4.log 2>&1
}
pmc r02zc 1024 1658 2048 40 3 && python3 tools/pmc_dw.py r02zc 1024 1658 2048 0 ae > gpurun_out/r02zc_pmc.txt 2>&1 && \
pmc r02zd 4096 1658 2048 40 0 && python3 tools/pmc_dw.py r02zd 4096 1658 2048 0 vib_ae > gpurun_out/r02zd_pmc.txt 2>&1
cp profiles/r02zc_pmc_dw.json profiles/r02zd_pmc_dw.json gpurun_out/ 2>/dev/null || true
