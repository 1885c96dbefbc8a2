set -uo pipefail
bash tools/gpu_lib_ab.sh r5w "wd or widedeep or wide or Wide" widedeep "--steps 5 --warmup 1" cascade cascade2 cascade3 cascade cascade2 cascade3 && bash tools/gpu_kstats.sh r5w_wd --workload widedeep --steps 5 --warmup 1
