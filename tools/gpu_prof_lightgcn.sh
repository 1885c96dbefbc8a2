set -uo pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/${TAG:-r4j}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for w in lightgcn lightgcn128; do
  echo "== prof $w $(date +%T)"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$w" -o $w -- python3 "$ROOT/bench.py" --workload $w --profile-only > "$OUT/prof_$w.log" 2>&1 || { echo "rocprof $w failed"; tail -5 "$OUT/prof_$w.log"; exit 1; }
  grep '^{' "$OUT/prof_$w.log" | tail -1 | cut -c1-600
done
cd $ROOT
for w in lightgcn lightgcn128; do bash tools/pmc_profile.sh $w gpurun_out/r4j_pmc_$w || exit 1; done
echo ok
