set -uo pipefail
mkdir -p gpurun_out/abl
for v in 0 101 102 103 104; do
  timeout -k 10 200 python bench.py --workload widedeep --steps 4 --warmup 1 --no-cpu-baseline --scan-users $v > gpurun_out/abl/wd_$v.json 2>gpurun_out/abl/wd_$v.err || { echo "fail $v"; tail gpurun_out/abl/wd_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abl/wd_$v.json'));print($v, d['roofline']['avg_kernel_ms'], d['ms_per_step'])"
done
