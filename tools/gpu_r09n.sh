# round-5 call: full GPU suite (teacher-forced records), persistent-grid A/B,
# then the c2 / c3 in-step schedule study (side-stream hold, BN apply mode)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
MMAD_TEACHER_OUT=gpurun_out/r09n_teacher timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s -rf --timeout 300 --timeout-method thread > gpurun_out/r09n_suite.log 2>&1
echo "suite rc=$?"
grep -q "segmentation\|Aborted\|core dumped" gpurun_out/r09n_suite.log && exit 1
timeout -k 10 300 python -u tools/tile_ab.py 65536 1+1p+6+6p 9+0 3 fwd > gpurun_out/r09n_persist_ab.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/tile_ab.py 65536 1+1p+6+6p 9 3 score >> gpurun_out/r09n_persist_ab.log 2>&1 || exit 1
bash tools/gpu_run.sh r09n bench:--config,c5,--no-cpu-baseline,--steps,5,--warmup,2 bench:--config,c5,--no-cpu-baseline,--steps,5,--warmup,2,--tune,persist=1 bench:--config,c2,--no-cpu-baseline,--no-probe bench:--config,c2,--no-cpu-baseline,--no-probe,--tune,side_hold=1 bench:--config,c2,--no-cpu-baseline,--no-probe,--tune,bn_mode=0 bench:--config,c3,--no-cpu-baseline,--no-probe bench:--config,c3,--no-cpu-baseline,--no-probe,--tune,side_hold=1 prof:--config,c2,--no-cpu-baseline,--no-probe,--steps,40 prof:--config,c2,--no-cpu-baseline,--no-probe,--steps,40,--tune,side_hold=1 prof:--config,c2,--no-cpu-baseline,--no-probe,--steps,40,--tune,bn_mode=0
