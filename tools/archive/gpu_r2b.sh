#!/bin/bash
# NCF certified path on personalised weights + serve-path B=1 latency (NCF, LightGCN cached).
set -uo pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 300 python bench.py --weights personal --no-cpu-baseline > gpurun_out/r2b/personal.out 2> gpurun_out/r2b/personal.err && tail -1 gpurun_out/r2b/personal.out &&
timeout -k 10 300 python bench.py --latency --steps 200 > gpurun_out/r2b/lat_ncf.out 2> gpurun_out/r2b/lat_ncf.err && cat gpurun_out/r2b/lat_ncf.out &&
timeout -k 10 300 python bench.py --latency --workload lightgcn --steps 200 > gpurun_out/r2b/lat_lgcn.out 2> gpurun_out/r2b/lat_lgcn.err && cat gpurun_out/r2b/lat_lgcn.out
