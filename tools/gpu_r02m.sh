# fused BN v3 (arrive before the a store, a kept in registers): tests, c2/c3 per BN mode, c2 traces mode 0 and 2
set -o pipefail
T=${1:-r02m}
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-probe --steps 100 --warmup 20"
timeout -k 10 300 python -u -m pytest -q -rA --timeout 120 --timeout-method thread tests/test_gpu_bn_fused.py > gpurun_out/${T}_pytest_bnf.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/${T}_pytest_bnf.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in 2 0 1; do
  MMAD_BN_MODE=$m timeout -k 10 100 $B > gpurun_out/${T}_c2_m$m.log 2>&1 || exit 3
  MMAD_BN_MODE=$m timeout -k 10 150 $B --config c3 > gpurun_out/${T}_c3_m$m.log 2>&1 || exit 3
done
MMAD_BN_MODE=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2_m2 -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 50 --warmup 10 > gpurun_out/${T}_prof_c2_m2.log 2>&1 && \
MMAD_BN_MODE=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2_m0 -o run -- python3 bench.py --no-cpu-baseline --no-probe --steps 50 --warmup 10 > gpurun_out/${T}_prof_c2_m0.log 2>&1
