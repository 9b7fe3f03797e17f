# C5 scoring: batch size sweep (graph replay), current code.
set -o pipefail
T=${1:-r02cc}
mkdir -p gpurun_out && export TMPDIR=/tmp
for b in 131072 262144 65536; do
  timeout -k 10 200 python -u bench_score.py --no-cpu-baseline --batch $b > /tmp/s.txt 2>&1 || { cat /tmp/s.txt > gpurun_out/${T}_err.txt; exit 1; }
  grep '^{' /tmp/s.txt > gpurun_out/${T}_b$b.json
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_b$b.json')); print('batch $b', d['value'], d['ms_total'], d.get('eager_ms_total', d.get('eager')))" >> gpurun_out/${T}_sum.txt
done
