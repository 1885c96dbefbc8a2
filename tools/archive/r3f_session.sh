set -uo pipefail
OUT=gpurun_out/r3f; mkdir -p $OUT
bash tools/archive/r3e_session.sh || exit 1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "dot or mf or lightgcn or prefilter" > $OUT/tests_dsA.out 2>&1 || { echo "dsA tests failed"; grep -E "FAILED|Error|assert" $OUT/tests_dsA.out | head; tail -20 $OUT/tests_dsA.out; exit 1; }
tail -1 $OUT/tests_dsA.out
HNM_LIB_PATH=$PWD/tools/bin/libhnm_dsB.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "dot or mf or prefilter" > $OUT/tests_dsB.out 2>&1 || { echo "dsB tests failed"; grep -E "FAILED|Error|assert" $OUT/tests_dsB.out | head; tail -20 $OUT/tests_dsB.out; exit 1; }
tail -1 $OUT/tests_dsB.out
bash tools/gpu_lib_ab.sh r3f_mf - mf "" prod dsA dsB prod dsA dsB || exit 1
echo ok
