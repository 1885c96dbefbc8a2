set -uo pipefail
OUT=gpurun_out/r3c; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.out 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/tests.out | head; tail -30 $OUT/tests.out; exit 1; }
tail -1 $OUT/tests.out
for t in prod short0 short64 short256; do for dd in 64 128; do
  HNM_LIB_PATH=$PWD/tools/bin/libhnm_$t.so timeout -k 10 200 python tools/spmm_halves.py --d $dd > $OUT/h_${t}_$dd.out 2>&1 || { echo "halves $t failed"; tail -5 $OUT/h_${t}_$dd.out; exit 1; }
  echo "$t d=$dd $(grep -E '^(users|items|layer)' $OUT/h_${t}_$dd.out | tr '\n' ' ')"
done; done
bash tools/gpu_lib_ab.sh r3c_ncf - ncf "" prod hybrid prod hybrid || exit 1
bash tools/gpu_lib_ab.sh r3c_lgcn - lightgcn "" prod short0 || exit 1
echo ok
