# Kernel stats (rocprofv3 --kernel-trace --stats, SQLite summarised by tools/prof_db.py) of the default c2 / c3 bench.
set -o pipefail
T=${1:-r02br}
mkdir -p gpurun_out && export TMPDIR=/tmp
for c in c2 c3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p_$c -o run -- python3 bench.py --config $c --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/${T}_bench_$c.log 2>&1 || exit 1
  python3 tools/prof_db.py $(find /tmp/p_$c -name "*.db" | head -1) --csv gpurun_out/${T}_kernel_stats_$c.csv > gpurun_out/${T}_kstats_$c.txt 2>&1 && python3 tools/prof_db.py $(find /tmp/p_$c -name "*.db" | head -1) --by-grid --csv gpurun_out/${T}_kernel_stats_bygrid_$c.csv > gpurun_out/${T}_kstats_bygrid_$c.txt 2>&1
  find /tmp/p_$c -name "*.csv" -exec cp {} gpurun_out/ \; || true
done
