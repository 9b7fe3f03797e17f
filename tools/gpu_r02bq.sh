# Round-2 final state: full GPU suite, smoke, c2 (with CPU baseline) / c3 bench lines, c2/c3 kernel stats + timelines.
set -o pipefail
T=${1:-r02bq}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench_c2.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/${T}_bench_c3.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 30 --warmup 10 > gpurun_out/${T}_prof_c2.log 2>&1 || exit 1
python3 tools/prof_step.py $(find gpurun_out/${T}_prof_c2 -name "*.db" | head -1) --last 20 > gpurun_out/${T}_timeline_c2.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c3 -o run -- python3 bench.py --config c3 --no-cpu-baseline --no-probe --steps 30 --warmup 10 > gpurun_out/${T}_prof_c3.log 2>&1 || exit 1
python3 tools/prof_step.py $(find gpurun_out/${T}_prof_c3 -name "*.db" | head -1) --last 20 > gpurun_out/${T}_timeline_c3.txt 2>&1
find gpurun_out/${T}_prof_c2 gpurun_out/${T}_prof_c3 -name "*.db" -delete
