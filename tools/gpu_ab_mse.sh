set -o pipefail
O=gpurun_out; L=icra2021_multimodal_ad_amd/libmmad.so
cp $L /tmp/libmmad_build.so
for lib in old new old new; do
  cp tools/ab/libmmad_$lib.so $L
  echo "== $lib" >> $O/r10h_mse_ab.jsonl
  timeout -k 10 120 python3 tools/mse_probe.py 4096 2,1,0 2>>$O/r10h_err.log | grep -v amdgpu >> $O/r10h_mse_ab.jsonl || exit 1
  timeout -k 10 120 python3 tools/mse_probe.py 1024 3,0,2 2>>$O/r10h_err.log | grep -v amdgpu >> $O/r10h_mse_ab.jsonl || exit 1
done
cp /tmp/libmmad_build.so $L
