# One GPU call: GPU tests, the default bench line, a rocprofv3 kernel trace of
# the bench and the PMC passes for the roofline GEMM (separate passes).
# Usage on the box: bash tools/gpu_profile_round.sh <tag>
set -o pipefail
T=${1:-rXX}
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --no-cpu-baseline --steps 100 > gpurun_out/${T}_prof.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_pmc_fetch -o run -- python3 tools/gemm_one.py fwd 0 1024 40 > gpurun_out/${T}_pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_pmc_write -o run -- python3 tools/gemm_one.py fwd 0 1024 40 > gpurun_out/${T}_pmc2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${T}_pmc_hit -o run -- python3 tools/gemm_one.py fwd 0 1024 40 > gpurun_out/${T}_pmc3.log 2>&1
