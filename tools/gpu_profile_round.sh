mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01j_pytest.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 300 > gpurun_out/r01j_bench_pair.log 2>&1 && \
MMAD_SHADOW_PAIR=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 300 > gpurun_out/r01j_bench_nopair.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r01j_prof -o run -- python3 bench.py --no-cpu-baseline --steps 100 > gpurun_out/r01j_prof.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r01j_pmc_fetch -o run -- python3 tools/gemm_one.py fwd 0 1024 40 > gpurun_out/r01j_pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r01j_pmc_write -o run -- python3 tools/gemm_one.py fwd 0 1024 40 > gpurun_out/r01j_pmc2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/r01j_pmc_hit -o run -- python3 tools/gemm_one.py fwd 0 1024 40 > gpurun_out/r01j_pmc3.log 2>&1
