set -o pipefail
TAG=${1:-r}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/test_gpu_prefilter.py -x -q -s > gpurun_out/$TAG/prefilter.out 2>&1 || { tail -30 gpurun_out/$TAG/prefilter.out; exit 1; }
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/$TAG/tests.out 2>&1 || { tail -30 gpurun_out/$TAG/tests.out; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/ncf.json 2> gpurun_out/$TAG/ncf.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --exact > gpurun_out/$TAG/ncf_exact.json 2> gpurun_out/$TAG/ncf_exact.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_ncf -o ncf -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_ncf.log 2>&1 || exit 1
echo done
