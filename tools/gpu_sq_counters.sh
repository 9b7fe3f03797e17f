mkdir -p gpurun_out && export TMPDIR=/tmp && \
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" && \
C2="SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU" && \
timeout -s KILL 60 rocprofv3 --pmc $C1 -d gpurun_out/r01m_sq_bd1 -o run -- python3 tools/gemm_one.py bwd_data 9 1024 20 > gpurun_out/r01m_sq1.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc $C1 -d gpurun_out/r01m_sq_f1 -o run -- python3 tools/gemm_one.py fwd 0 1024 20 > gpurun_out/r01m_sq2.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc $C2 -d gpurun_out/r01m_sq_bd2 -o run -- python3 tools/gemm_one.py bwd_data 9 1024 20 > gpurun_out/r01m_sq3.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc $C2 -d gpurun_out/r01m_sq_f2 -o run -- python3 tools/gemm_one.py fwd 0 1024 20 > gpurun_out/r01m_sq4.log 2>&1
