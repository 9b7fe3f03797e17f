# dW+Adam PMC passes (cold Adam state), C3 PMC passes over the bench, defaults bench c2/c3
set -o pipefail
T=${1:-r02p}
mkdir -p gpurun_out && export TMPDIR=/tmp
D="python3 tools/dw_one.py 1024 1658 2048 40 3"
timeout -k 10 100 python -u tools/dw_one.py 1024 1658 2048 40 3 > gpurun_out/${T}_dwone.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_pmc_fetch -o run -- $D > gpurun_out/${T}_pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_pmc_write -o run -- $D > gpurun_out/${T}_pmc2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${T}_pmc_hit -o run -- $D > gpurun_out/${T}_pmc3.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${T}_pmc_mfma -o run -- $D > gpurun_out/${T}_pmc4.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_dwone -o run -- $D > gpurun_out/${T}_prof_dwone.log 2>&1 && \
C="python3 bench.py --config c3 --no-cpu-baseline --no-probe --steps 20 --warmup 5" && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_c3pmc_fetch -o run -- $C > gpurun_out/${T}_c3pmc1.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_c3pmc_write -o run -- $C > gpurun_out/${T}_c3pmc2.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${T}_c3pmc_mfma -o run -- $C > gpurun_out/${T}_c3pmc3.log 2>&1 && \
timeout -k 10 150 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_c2.log 2>&1 && \
timeout -k 10 150 python -u bench.py --config c3 --no-cpu-baseline --steps 100 > gpurun_out/${T}_c3.log 2>&1
