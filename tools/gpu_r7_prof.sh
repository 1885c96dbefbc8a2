set -uo pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r7m; mkdir -p $OUT
HNM_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --workload lightgcn128 --steps 5 --warmup 2 > $OUT/bench_2rank.out 2> $OUT/bench_2rank.err || { echo 2rank failed; tail -20 $OUT/bench_2rank.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
for w in ncf lightgcn widedeep mf ncf_deep; do
  extra=""
  [ $w = widedeep ] && extra="--steps 3 --warmup 1"
  echo "== prof $w $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$w" -o $w -- python3 "$ROOT/bench.py" --workload $w $extra --profile-only > "$OUT/prof_$w.log" 2>&1 || { echo "rocprof $w failed"; exit 1; }
done
echo ok
