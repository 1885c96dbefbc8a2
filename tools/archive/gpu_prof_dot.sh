# rocprofv3 kernel stats of the dot workloads (run on the GPU box)
set -o pipefail
TAG=${1:-r}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for w in lightgcn mf; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/$TAG/prof_$w -o $w -- python3 $ROOT/bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $ROOT/gpurun_out/$TAG/prof_$w.log 2>&1 || exit 1
done
echo done
