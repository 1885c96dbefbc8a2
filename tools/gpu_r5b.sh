set -uo pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 600 python -u -m pytest tests -v -s -m gpu --timeout 300 --timeout-method thread -k "strided_sample_gate" > gpurun_out/r5c/tests.out 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r5c/tests.out | head -20; tail -30 gpurun_out/r5c/tests.out; exit 1; }
grep -E "NCF |passed|failed" gpurun_out/r5c/tests.out | tail -20
for wt in personal norms student_t; do timeout -k 10 240 python bench.py --workload ncf --weights $wt --profile-only > gpurun_out/r5c/ncf_$wt.json 2> gpurun_out/r5c/ncf_$wt.err || exit 1; done
timeout -k 10 240 python bench.py --workload ncf --profile-only > gpurun_out/r5c/ncf_init.json 2> gpurun_out/r5c/ncf_init.err || exit 1
for f in ncf_personal ncf_norms ncf_student_t ncf_init; do python -c "
import json
d=json.loads(open('gpurun_out/r5c/$f.json').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_kernel_ms'], d.get('prefilter'))"; done
