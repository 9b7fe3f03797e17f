# A/B of two prebuilt libraries (tools/ab/libmmad_{old,new}.so swapped into
# the package between runs) on c3 / c2, then a c3 sweep of the dW split rule
set -o pipefail
O=gpurun_out
L=icra2021_multimodal_ad_amd/libmmad.so
cp $L /tmp/libmmad_build.so
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_gemm.py > $O/r0ax_tests.log 2>&1 || exit 1
for lib in old new old new; do
  cp tools/ab/libmmad_$lib.so $L
  echo "== $lib" >> $O/r0ax_ab.jsonl
  timeout -k 10 200 python3 bench.py --no-cpu-baseline 2>>$O/r0ax_err.log | tail -1 >> $O/r0ax_ab.jsonl || exit 1
done
cp /tmp/libmmad_build.so $L
for t in "" "splitk_dw_blocks=64" "splitk_dw_blocks=128" "splitk_dw_blocks=256" "splitk_dw_blocks=512" "" "splitk_dw_blocks=256 splitk_dw_min_stages=4"; do
  args=""; for kv in $t; do args="$args --tune $kv"; done
  echo "== $t" >> $O/r0ax_sweep.jsonl
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-c2 $args 2>>$O/r0ax_err.log | tail -1 >> $O/r0ax_sweep.jsonl || exit 1
done
