# rocprofv3 kernel stats of one bench workload (run on the GPU box): tools/gpu_prof.sh <tag> <workload> [bench args]
set -o pipefail
TAG=${1:-r}; W=${2:-ncf}; shift 2 || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/$TAG/prof_$W -o $W -- python3 $ROOT/bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline "$@" > $ROOT/gpurun_out/$TAG/prof_$W.log 2>&1
