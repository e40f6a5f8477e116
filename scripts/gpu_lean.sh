# lean_kernel parity + the general GPU parity suite + one bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/lean
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lean.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_lean.log 2>&1
rc=$?
tail -25 $OUT/pytest_lean.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_all.log 2>&1
rc=$?
tail -5 $OUT/pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
