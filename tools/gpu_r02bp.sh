# Tail pair launch (MMAD_DW_PAIR): full GPU suite (GEMM body refactor), then c2/c3 bench pair on/off.
set -o pipefail
T=${1:-r02bp}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
for rep in 1 2; do for p in 1 0; do for c in c2 c3; do
  MMAD_DW_PAIR=$p timeout -k 10 150 python -u bench.py --no-cpu-baseline --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; exit 1; }
  tail -1 /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('pair=$p $c', d['ms_per_step'], r['avg_us'], r['frac'], r['kernel'][:60])" >> gpurun_out/${T}_sum.txt
done; done; done
