# NCF certified-scan tuning session: parity tests of the pre-filter, then bench variants.
set -o pipefail
TAG=${1:-r}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/test_gpu_prefilter.py tests/test_gpu_parity.py -x -q -s -k "ncf or prefilter or bound" > gpurun_out/$TAG/prefilter.out 2>&1 || { tail -30 gpurun_out/$TAG/prefilter.out; exit 1; }
for v in ${VARIANTS:-1 2 3 4}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --scan-users $v > gpurun_out/$TAG/ncf_u$v.json 2> gpurun_out/$TAG/ncf_u$v.err || exit 1
done
echo done
