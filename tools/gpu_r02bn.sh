# GEMM main-loop schedule variants (MMAD_LOOP_VARIANT builds under tools/variants): per-GEMM timing, then c2/c3 bench.
set -o pipefail
T=${1:-r02bn}
mkdir -p gpurun_out && export TMPDIR=/tmp
for v in 0 1 2 3; do
  if [ $v = 0 ]; then L=icra2021_multimodal_ad_amd/libmmad.so; else L=tools/variants/libmmad_v$v.so; fi
  for spec in "fwd 0 4096 1" "fwd 0 4096 2" "fwd 0 16384 2" "fwd 0 1024 3" "bwd_data 1 4096 1" "bwd_data 0 1024 3" "bwd_w 0 1024 3" "bwd_w 0 4096 0"; do
    MMAD_LIB=$L timeout -k 10 60 python -u tools/gemm_time.py $spec > /tmp/o.txt 2>&1 || { cat /tmp/o.txt >> gpurun_out/${T}_time.txt; exit 1; }
    echo "v$v $(tail -1 /tmp/o.txt)" >> gpurun_out/${T}_time.txt
  done
done
for v in 0 1 2 3; do
  if [ $v = 0 ]; then L=icra2021_multimodal_ad_amd/libmmad.so; else L=tools/variants/libmmad_v$v.so; fi
  for c in c2 c3; do
    MMAD_LIB=$L timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt >> gpurun_out/${T}_bench.txt; exit 1; }
    tail -1 /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('v$v $c', d['ms_per_step'])" >> gpurun_out/${T}_bench.txt
  done
done
