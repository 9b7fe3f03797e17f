# Streamed Adam: tile / consumer-grid sweep at c2 and c3, then the c2 kernel timeline.
set -o pipefail
T=${1:-r02bf}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --steps 300"
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 150 $B > gpurun_out/${T}_${tag}_c2.log 2>&1 || return 1
  env "$@" timeout -k 10 150 $B --config c3 > gpurun_out/${T}_${tag}_c3.log 2>&1 || return 1
  for c in c2 c3; do
    tail -1 gpurun_out/${T}_${tag}_${c}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $c', d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['frac'])" >> gpurun_out/${T}_sum.txt
  done
}
run off MMAD_ADAM_STREAM=0 && run t3g512 MMAD_ADAM_STREAM=1 && run t3g256 MMAD_ADAM_STREAM=1 MMAD_ADAM_STREAM_GRID=256 && \
run tautog512 MMAD_ADAM_STREAM=1 MMAD_ADAM_STREAM_TILE=-1 && run t4g512 MMAD_ADAM_STREAM=1 MMAD_ADAM_STREAM_TILE=4 && \
MMAD_ADAM_STREAM=1 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/ks -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 30 --warmup 10 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/prof_step.py $(find /tmp/ks -name "*.db" | head -1) --last 20 > gpurun_out/${T}_timeline.txt 2>&1
