# c3 kernel timeline (current defaults) and HBM traffic of the BN kernels (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
T=${1:-r02bh}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/kc3 -o run -- python3 bench.py --config c3 --no-cpu-baseline --no-probe --steps 30 --warmup 10 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/prof_step.py $(find /tmp/kc3 -name "*.db" | head -1) --last 20 > gpurun_out/${T}_timeline_c3.txt 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf -o run -- python3 bench.py --config c3 --no-cpu-baseline --no-probe --steps 10 --warmup 3 > gpurun_out/${T}_pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw -o run -- python3 bench.py --config c3 --no-cpu-baseline --no-probe --steps 10 --warmup 3 > gpurun_out/${T}_pmc2.log 2>&1 && \
python3 tools/pmc_by_kernel.py /tmp/pf /tmp/pw > gpurun_out/${T}_pmc_bn.txt 2>&1
