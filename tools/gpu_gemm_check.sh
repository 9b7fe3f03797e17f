mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01n_pytest.log 2>&1 && \
timeout -k 10 120 python -u tools/gemm_probe.py bwd_data 9 > gpurun_out/r01n_probe_bd9.log 2>&1 && \
timeout -k 10 120 python -u tools/gemm_probe.py bwd_w 9 > gpurun_out/r01n_probe_bw9.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/r01n_sq_bd1 -o run -- python3 tools/gemm_one.py bwd_data 9 1024 20 > gpurun_out/r01n_sq1.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 300 > gpurun_out/r01n_bench.log 2>&1
