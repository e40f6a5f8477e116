# GPU tests (optionally a subset: TESTS="tests/test_gpu_lean.py ...") then a short
# bench line.  Usage on the box:  TAG=x bash scripts/gpu_quick.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -8 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err; exit $rc
