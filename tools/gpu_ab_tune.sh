# A/B of one tune-table knob's values on the same library, alternating rounds
# Usage: bash tools/gpu_ab_tune.sh <tag> <knob> "<v1> <v2> ..." [rounds=2] [bench args...]
set -o pipefail
T=$1; K=$2; VALS=$3; R=${4:-2}; shift 4
O=gpurun_out
for r in $(seq $R); do
  for v in $VALS; do
    echo "== $K=$v" >> $O/${T}_tune_ab.jsonl
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --tune $K=$v "$@" 2>>$O/${T}_err.log | tail -1 >> $O/${T}_tune_ab.jsonl || exit 1
  done
done
