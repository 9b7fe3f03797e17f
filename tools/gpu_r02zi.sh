# End-of-session check on the final commit: full GPU suite, smoke, default bench (c2 with CPU baseline), c3.
set -o pipefail
T=${1:-r02zi}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench_c2.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/${T}_bench_c3.log 2>&1
