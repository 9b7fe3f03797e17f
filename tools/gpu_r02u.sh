# DP schedule overhead on one GPU (loopback exchange), c2 and c3 shapes; C5 scoring bench refresh
set -o pipefail
T=${1:-r02u}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u tools/dp_overhead.py 50 > gpurun_out/${T}_dp.log 2>&1 && \
timeout -k 10 300 python -u bench_score.py > gpurun_out/${T}_score.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_score -o run -- python3 bench_score.py --no-cpu-baseline > gpurun_out/${T}_prof_score.log 2>&1
