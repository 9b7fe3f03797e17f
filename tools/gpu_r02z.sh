set -o pipefail
T=${1:-r02z}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hsr_ingest.py tests/test_hsr.py -q -rA --timeout 200 --timeout-method thread > gpurun_out/${T}_ingest.log 2>&1
