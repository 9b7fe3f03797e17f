set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for v in "0 0 0 20 1024 8 0 noraw:fused" "8 0 1 20 1024 8 1024 noraw:each"; do
  a=${v%%:*}; t=${v##*:}
  timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/r0ay_$t -o run -- python3 tools/dp_probe.py $a > $O/r0ay_$t.log 2>&1 || exit 1
  python3 tools/prof_step.py "$(find /tmp/r0ay_$t -name '*.db' | head -1)" --last 20 > $O/r0ay_timeline_c2_$t.txt || exit 1
done
