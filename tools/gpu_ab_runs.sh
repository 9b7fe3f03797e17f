# A/B of two prebuilt libraries (tools/ab/libmmad_{old,new}.so), N alternating
# bench processes each (every process autotunes anew)
# Usage: bash tools/gpu_ab_runs.sh <tag> <n> [bench args...]
set -o pipefail
T=$1; N=$2; shift 2
O=gpurun_out
L=icra2021_multimodal_ad_amd/libmmad.so
cp $L /tmp/libmmad_build.so
for i in $(seq $N); do
  for lib in old new; do
    cp tools/ab/libmmad_$lib.so $L
    echo "== $lib" >> $O/${T}_ab.jsonl
    timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" 2>>$O/${T}_err.log | tail -1 >> $O/${T}_ab.jsonl || exit 1
  done
done
cp /tmp/libmmad_build.so $L
