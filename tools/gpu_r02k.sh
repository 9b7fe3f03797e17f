# fused train-mode BN: its tests, the whole gpu suite (default mode), c2/c3 bench per BN mode, c2 kernel trace (mode 2)
set -o pipefail
T=${1:-r02k}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --steps 100 --warmup 20"
timeout -k 10 300 python -u -m pytest -q -rA --timeout 120 --timeout-method thread tests/test_gpu_bn_fused.py "tests/test_gpu_vib_full.py::test_vib_ae_full_size_fp32_matches_oracle" > gpurun_out/${T}_pytest_bnf.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_pytest_bnf.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
MMAD_BN_MODE=2 timeout -k 10 100 $B > gpurun_out/${T}_c2_bnf.log 2>&1 && \
MMAD_BN_MODE=0 timeout -k 10 100 $B > gpurun_out/${T}_c2_apply.log 2>&1 && \
timeout -k 10 100 $B > gpurun_out/${T}_c2_fold.log 2>&1 && \
MMAD_BN_MODE=2 timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3_bnf.log 2>&1 && \
timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3_fold.log 2>&1 && \
MMAD_BN_MODE=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/${T}_prof_c2.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
