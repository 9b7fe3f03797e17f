set -o pipefail
T=${1:-r02ag}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-probe --steps 200 --warmup 20"
run() { name=$1; shift; env "$@" timeout -k 10 150 $B $CFG > gpurun_out/${T}_${name}.log 2>&1; }
CFG=""
run c2_eager1 && run c2_graph1 MMAD_TRAIN_GRAPH=1 && run c2_eager2 && run c2_graph2 MMAD_TRAIN_GRAPH=1 && \
CFG="--config c3" && run c3_eager && run c3_graph MMAD_TRAIN_GRAPH=1
