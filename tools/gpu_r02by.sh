# Final state after the schedule changes: smoke, c2 (CPU baseline) / c3 bench lines, kernel stats by grid, step timelines.
set -o pipefail
T=${1:-r02by}
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench_c2.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/${T}_bench_c3.log 2>&1 || exit 1
for c in c2 c3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p_$c -o run -- python3 bench.py --config $c --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/${T}_benchprof_$c.log 2>&1 || exit 1
  D=$(find /tmp/p_$c -name "*.db" | head -1)
  python3 tools/prof_db.py $D --by-grid --csv gpurun_out/${T}_kernel_stats_bygrid_$c.csv > gpurun_out/${T}_kstats_bygrid_$c.txt 2>&1 && \
  python3 tools/prof_step.py $D --last 20 > gpurun_out/${T}_timeline_$c.txt 2>&1 || exit 1
done
