# kernel trace of the c3 step (VIB-AE, 4096 windows): per-kernel breakdown
set -o pipefail
T=${1:-r02aa}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c3 -o run -- python3 bench.py --config c3 --no-cpu-baseline --no-probe --steps 30 --warmup 10 > gpurun_out/${T}_prof_c3.log 2>&1
