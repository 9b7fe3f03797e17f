# bench.py --gpus 2 harness on one GPU (both ranks on cuda:0 over gloo): spawn, rendezvous, timing, n1_same_workload, probe, report.
set -o pipefail
T=${1:-r02zg}
mkdir -p gpurun_out && export TMPDIR=/tmp
MMAD_BENCH_SHARED_GPU=1 timeout -k 10 150 python -u bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_n2.log 2>&1
