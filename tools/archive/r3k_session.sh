set -uo pipefail
OUT=gpurun_out/r3k; mkdir -p $OUT
HNM_LIB_PATH=$PWD/tools/bin/libhnm_p3.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "wd_ or widedeep" > $OUT/tests_p3.out 2>&1 || { echo "p3 tests failed"; grep -E "FAILED|Error|assert" $OUT/tests_p3.out | head -20; tail -30 $OUT/tests_p3.out; exit 1; }
tail -1 $OUT/tests_p3.out
bash tools/gpu_lib_ab.sh r3k_wd - widedeep "--steps 5 --warmup 1" prod p3 prod p3 || exit 1
echo ok
