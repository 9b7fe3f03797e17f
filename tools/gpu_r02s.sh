set -o pipefail
T=${1:-r02s}
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench_launch > gpurun_out/${T}_launch.log 2>&1 && \
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 60 ./tools/ubench_launch >> gpurun_out/${T}_launch.log 2>&1 && \
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 60 ./tools/ubench_launch >> gpurun_out/${T}_launch.log 2>&1 && \
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 100 python -u bench.py --no-cpu-baseline --no-probe > gpurun_out/${T}_c2_devka.log 2>&1 && \
timeout -k 10 100 python -u bench.py --no-cpu-baseline --no-probe > gpurun_out/${T}_c2.log 2>&1
