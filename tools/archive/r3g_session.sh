set -uo pipefail
OUT=gpurun_out/r3g; mkdir -p $OUT
HNM_LIB_PATH=$PWD/tools/bin/libhnm_wd2.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "wd_ or widedeep" > $OUT/tests_wd2.out 2>&1 || { echo "wd2 tests failed"; grep -E "FAILED|Error|assert" $OUT/tests_wd2.out | head -20; tail -30 $OUT/tests_wd2.out; exit 1; }
tail -1 $OUT/tests_wd2.out
HNM_LIB_PATH=$PWD/tools/bin/libhnm_dsC.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "dot or mf or prefilter" > $OUT/tests_dsC.out 2>&1 || { echo "dsC tests failed"; grep -E "FAILED|Error|assert" $OUT/tests_dsC.out | head; tail -20 $OUT/tests_dsC.out; exit 1; }
tail -1 $OUT/tests_dsC.out
bash tools/gpu_lib_ab.sh r3g_wd - widedeep "--steps 5 --warmup 1" prod wd2 wd1 prod wd2 || exit 1
bash tools/gpu_lib_ab.sh r3g_mf - mf "" dsB dsC dsB dsC || exit 1
bash tools/gpu_lib_ab.sh r3g_lg - lightgcn "" prod dsB dsC || exit 1
echo ok
