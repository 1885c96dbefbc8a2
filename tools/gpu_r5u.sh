set -uo pipefail
bash tools/gpu_lib_ab.sh r5z "wd or widedeep or wide or Wide" widedeep "--steps 5 --warmup 1" cascade3 cascade5 cascade3 cascade5 && bash tools/gpu_kstats.sh r5z_wd --workload widedeep --steps 5 --warmup 1
