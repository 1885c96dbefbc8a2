set -uo pipefail
OUT=gpurun_out/r3e; mkdir -p $OUT
HNM_LIB_PATH=$PWD/tools/bin/libhnm_wd1.so timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "wd_ or widedeep" > $OUT/tests_wd1.out 2>&1 || { echo "wd1 tests failed"; grep -E "FAILED|Error|assert" $OUT/tests_wd1.out | head -20; tail -30 $OUT/tests_wd1.out; exit 1; }
tail -1 $OUT/tests_wd1.out
bash tools/gpu_lib_ab.sh r3e_ab - widedeep "--steps 5 --warmup 1" prod wd1 prod wd1 || exit 1
echo ok
