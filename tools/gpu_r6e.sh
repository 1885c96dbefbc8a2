set -uo pipefail
bash tools/gpu_lib_ab.sh r6e - mf "--steps 50 --warmup 5" dbase dq3 dq4 dbase dq3 dq4 dbase dq3 dq4
