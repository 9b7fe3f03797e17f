# A/B of two prebuilt libraries (tools/ab/libmmad_{old,new}.so swapped into
# the package between runs), alternating, then a kernel trace of the new one
# Usage: bash tools/gpu_ab_lib.sh <tag> [bench args...]
set -o pipefail
T=$1; shift
O=gpurun_out
L=icra2021_multimodal_ad_amd/libmmad.so
export TMPDIR=/tmp
cp $L /tmp/libmmad_build.so
for lib in old new old new old new; do
  cp tools/ab/libmmad_$lib.so $L
  echo "== $lib" >> $O/${T}_ab.jsonl
  timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" 2>>$O/${T}_err.log | tail -1 >> $O/${T}_ab.jsonl || exit 1
done
cp tools/ab/libmmad_new.so $L
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/${T}_prof -o run -- python3 bench.py --no-c2 --no-cpu-baseline --steps 20 --soak-s 0.5 > $O/${T}_prof.log 2>&1 || exit 1
python3 tools/prof_step.py "$(find /tmp/${T}_prof -name '*.db' | head -1)" --last 20 > $O/${T}_timeline.txt || exit 1
cp /tmp/libmmad_build.so $L
