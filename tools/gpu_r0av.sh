set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dp.py > $O/r0av_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/dp_overhead.py 50 4096 > $O/r0av_dp_overhead.txt 2>> $O/r0av_err.log || exit 1
timeout -k 10 300 python3 tools/dp_overhead.py 50 1024 >> $O/r0av_dp_overhead.txt 2>> $O/r0av_err.log || exit 1
bash tools/gpu_pmc.sh r0av c3w c2w > $O/r0av_pmc.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/r0av_bench_c3.json 2> $O/r0av_bench_c3.err
