set -uo pipefail
bash tools/gpu_lib_ab.sh r6d - widedeep "--steps 5 --warmup 1" wbase w2wave wbase w2wave
