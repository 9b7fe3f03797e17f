set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for a in "0 0 0 50 4096" "8 0 1 50 4096 8 0" "8 0 1 50 4096 8 2048" "0 0 0 50 4096" "8 0 1 50 4096 8 0" "8 0 1 50 4096 8 2048" "0 0 0 50 1024" "8 0 1 50 1024 8 0" "8 0 1 50 1024 8 1024"; do
  timeout -k 10 120 python3 tools/dp_probe.py $a 2>>$O/r0au_err.log | grep -v amdgpu.ids >> $O/r0au_dp.txt || exit 1
done
for v in "0 0 0 20 4096 8 0 noraw:fused" "8 0 1 20 4096 8 0 noraw:bucket" "8 0 1 20 4096 8 2048 noraw:each"; do
  a=${v%%:*}; t=${v##*:}
  timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/r0au_$t -o run -- python3 tools/dp_probe.py $a > $O/r0au_$t.log 2>&1 || exit 1
  python3 tools/prof_step.py "$(find /tmp/r0au_$t -name '*.db' | head -1)" --last 20 > $O/r0au_timeline_$t.txt || exit 1
done
timeout -k 10 300 python3 bench.py --config c5 > $O/r0au_bench_c5.json 2> $O/r0au_bench_c5.err
