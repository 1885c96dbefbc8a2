set -uo pipefail
HNM_LIB_PATH=$PWD/tools/bin/libhnm_diag.so bash tools/gpu_kstats.sh r5y_diag --workload widedeep --steps 3 --warmup 1 --no-cpu-baseline && HNM_LIB_PATH=$PWD/tools/bin/libhnm_cascade3.so bash tools/gpu_kstats.sh r5y_base --workload widedeep --steps 3 --warmup 1 --no-cpu-baseline
