set -uo pipefail
bash tools/gpu_lib_ab.sh r6n - ncf "--steps 20 --warmup 3 --profile-only" cur pf cur pf cur pf
