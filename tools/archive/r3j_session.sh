set -uo pipefail
OUT=gpurun_out/r3j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "wd_ or widedeep" > $OUT/tests_wd4.out 2>&1 || { echo "wd4 tests failed"; grep -E "FAILED|Error|assert" $OUT/tests_wd4.out | head -20; tail -30 $OUT/tests_wd4.out; exit 1; }
tail -1 $OUT/tests_wd4.out
bash tools/gpu_lib_ab.sh r3j_wd - widedeep "--steps 5 --warmup 1" prod wd4 wd3 prod wd4 || exit 1
echo ok
