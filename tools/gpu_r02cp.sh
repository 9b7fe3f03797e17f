# Same-box A/B: the library at ad925cd (c3 0.939 on its box) vs the current one, c2 / c3.
set -o pipefail
T=${1:-r02cp}
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2 3; do for v in old new; do
  if [ $v = old ]; then L=tools/variants/libmmad_ad925cd.so; else L=icra2021_multimodal_ad_amd/libmmad.so; fi
  for c in c3 c2; do
    MMAD_LIB=$L timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-probe --steps 300 --config $c > /tmp/b.txt 2>&1 || { cat /tmp/b.txt > gpurun_out/${T}_err.txt; exit 1; }
    grep '^{' /tmp/b.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $c', d['ms_per_step'])" >> gpurun_out/${T}_sum.txt
  done
done; done
