# A probe script run under two prebuilt libraries (tools/ab/libmmad_{old,new}.so
# swapped into the package), alternating: bash tools/gpu_ab_probe.sh <tag> <script> [args...]
set -o pipefail
T=$1; shift
O=gpurun_out; L=icra2021_multimodal_ad_amd/libmmad.so
cp $L /tmp/libmmad_build.so
for lib in old new old new; do
  cp tools/ab/libmmad_$lib.so $L
  echo "== $lib" >> $O/${T}_probe_ab.jsonl
  timeout -k 10 200 python3 "$@" 2>>$O/${T}_err.log | grep -v amdgpu >> $O/${T}_probe_ab.jsonl || exit 1
done
cp /tmp/libmmad_build.so $L
