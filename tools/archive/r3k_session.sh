set -uo pipefail
OUT=gpurun_out/r3k; mkdir -p $OUT
for t in p3 lox lox3; do
HNM_LIB_PATH=$PWD/tools/bin/libhnm_$t.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "wd_ or widedeep" > $OUT/tests_$t.out 2>&1 || { echo "$t tests failed"; grep -E "FAILED|Error|assert" $OUT/tests_$t.out | head -20; tail -30 $OUT/tests_$t.out; exit 1; }
echo "$t $(tail -1 $OUT/tests_$t.out)"
done
bash tools/gpu_lib_ab.sh r3k_wd - widedeep "--steps 5 --warmup 1" prod p3 lox lox3 prod p3 lox lox3 || exit 1
echo ok
