# Per-call ping-pong schedule (shadow pair by default, ping from 4096 rows, dw_main 1) + ev_every 2: full suite, c2/c3 bench.
set -o pipefail
T=${1:-r02bw}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
for rep in 1 2; do for c in c2 c3; do
  timeout -k 10 150 python -u bench.py --no-cpu-baseline --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; exit 1; }
  grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['frac'])" >> gpurun_out/${T}_sum.txt
done; done
