set -o pipefail
T=${1:-r02ak}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bn_fused.py tests/test_gpu_vib_full.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 && \
B="python -u bench.py --no-cpu-baseline --no-probe --steps 200 --warmup 20 --config c3"
timeout -k 10 150 $B > gpurun_out/${T}_c3a.log 2>&1 && timeout -k 10 150 $B > gpurun_out/${T}_c3b.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/kc3 -o run -- python3 bench.py --config c3 --no-cpu-baseline --no-probe --steps 20 --warmup 5 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/prof_db.py /tmp/kc3/*/run_results.db > gpurun_out/${T}_kstats.txt 2>&1 || python3 tools/prof_db.py $(find /tmp/kc3 -name "*.db" | head -1) > gpurun_out/${T}_kstats.txt 2>&1
