# Streamed Adam on the main-stream tail (knob MMAD_ADAM_STREAM): equivalence tests, c2/c3 bench on/off.
set -o pipefail
T=${1:-r02bd}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_adam_stream.py tests/test_gpu_bn_fused.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --steps 300"
for st in 1 0 1 0; do
  MMAD_ADAM_STREAM=$st timeout -k 10 150 $B > gpurun_out/${T}_c2_s${st}.log 2>&1 || exit 1
  tail -1 gpurun_out/${T}_c2_s${st}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 stream=$st', d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['frac'])" >> gpurun_out/${T}_sum.txt
  MMAD_ADAM_STREAM=$st timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3_s${st}.log 2>&1 || exit 1
  tail -1 gpurun_out/${T}_c3_s${st}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 stream=$st', d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['frac'])" >> gpurun_out/${T}_sum.txt
done
