# PMC passes (one counter group per rocprofv3 run, each under its own limit)
# for the c5 roofline kernel (tools/score_one.py), summarised on the box by
# tools/pmc_score.py into gpurun_out/ (the per-pass databases are removed).
# Usage: bash tools/gpu_pmc_c5.sh <tag> [batch=65536]
set -o pipefail
T=$1; B=${2:-65536}
mkdir -p gpurun_out profiles && export TMPDIR=/tmp
for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "hit TCC_HIT_sum TCC_MISS_sum"; do
  set -- $p; n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc $* -d gpurun_out/${T}_pmc_$n -o run -- python3 tools/score_one.py $B 20 \
    > gpurun_out/${T}_pmc_$n.log 2>&1 || exit 1
  echo "[pmc] ${T}_pmc_$n ok"
done
python3 tools/pmc_score.py $T $B && cp profiles/${T}_pmc_score.json gpurun_out/
rc=$?
rm -rf gpurun_out/${T}_pmc_fetch/ gpurun_out/${T}_pmc_write/ gpurun_out/${T}_pmc_hit/
exit $rc
