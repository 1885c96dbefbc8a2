#!/bin/bash
# GPU session part 1: the full -m gpu suite and smoke() (outputs under gpurun_out/<tag>/).
#   bash tools/gpu_tests.sh <tag> [pytest -k expr]
set -uo pipefail
TAG=${1:-r}; KEXPR=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
args=(-u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread)
[ -n "$KEXPR" ] && args+=(-k "$KEXPR")
timeout -k 10 1000 python "${args[@]}" > "$OUT/tests.out" 2>&1
rc=$?
echo "tests rc=$rc" >> "$OUT/status.txt"
grep -E "FAILED|ERROR" "$OUT/tests.out" | head -20
tail -1 "$OUT/tests.out"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.out" 2>&1
rc2=$?
echo "smoke rc=$rc2" >> "$OUT/status.txt"
tail -3 "$OUT/smoke.out"
exit $(( rc > rc2 ? rc : rc2 ))
