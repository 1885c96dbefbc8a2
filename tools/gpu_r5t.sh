set -uo pipefail
bash tools/gpu_lib_ab.sh r5t "dot or mf or lightgcn" mf "--steps 50 --warmup 5" shallow deep shallow deep shallow deep && bash tools/gpu_lib_ab.sh r5t - lightgcn "--steps 20 --warmup 3" shallow deep && bash tools/gpu_kstats.sh r5t_ncf --workload ncf
