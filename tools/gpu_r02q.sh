# Adam-state prefetch in the dW epilogue + split-K combine / fused-dz register fixes: suite, benches, dW PMC
set -o pipefail
T=${1:-r02q}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
D="python3 tools/dw_one.py 1024 1658 2048 40 3"
timeout -k 10 150 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_c2.log 2>&1 && \
timeout -k 10 150 python -u bench.py --config c3 --no-cpu-baseline --steps 100 > gpurun_out/${T}_c3.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_dwone -o run -- $D > gpurun_out/${T}_prof_dwone.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_pmc_fetch -o run -- $D > gpurun_out/${T}_pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_pmc_write -o run -- $D > gpurun_out/${T}_pmc2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${T}_pmc_hit -o run -- $D > gpurun_out/${T}_pmc3.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${T}_pmc_mfma -o run -- $D > gpurun_out/${T}_pmc4.log 2>&1
