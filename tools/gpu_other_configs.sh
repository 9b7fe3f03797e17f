# Bench lines of the other BASELINE configurations (one GPU call).
# Usage on the box: T=<tag> bash tools/gpu_other_configs.sh
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline --dim 1728 > gpurun_out/${T}_bench_d1728.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline --batch 4096 > gpurun_out/${T}_bench_ae4096.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline --batch 4096 --model vib_ae > gpurun_out/${T}_bench_vib4096.log 2>&1 && \
timeout -k 10 300 python -u bench_score.py > gpurun_out/${T}_bench_score.log 2>&1
