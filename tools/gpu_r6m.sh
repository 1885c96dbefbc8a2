set -uo pipefail
OUT=gpurun_out/r6m; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "ncf or NCF or prefilter or stress or shard or rccl" --timeout 300 --timeout-method thread > $OUT/tests.out 2>&1; echo "tests rc=$?"; tail -2 $OUT/tests.out
for wt in init personal norms student_t; do
  timeout -k 10 300 python bench.py --workload ncf --weights $wt --profile-only > $OUT/ncf_$wt.out 2> $OUT/ncf_$wt.err || { echo "bench $wt failed"; tail -5 $OUT/ncf_$wt.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/ncf_$wt.out').read().strip().splitlines()[-1]); print('$wt', d['value'], d['ms_per_step'], d['roofline'].get('avg_kernel_ms'), d['prefilter']['candidates_per_row'], d['prefilter']['fallback_rows'])"
done
bash tools/gpu_kstats.sh r6m_norms --workload ncf --weights norms | head -4
