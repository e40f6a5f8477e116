# classification tables A/B (CLS2 vs FAST_OLD_CLS) and the tokenizer/fast-path GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cls}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fast.py tests/test_gpu_lean.py tests/test_gpu_parity.py tests/test_gpu_tokenizer.py tests/test_gpu_records.py tests/test_gpu_fastjoin.py tests/test_gpu_partials.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 420 python -u scripts/variant_bench.py base ${VARIANTS:-ocls} --rounds 3 --steps 10 > $OUT/c3.log 2>&1 || exit 1
tail -1 $OUT/c3.log
timeout -k 10 300 python -u scripts/variant_bench.py base ${VARIANTS:-ocls} --config 2 --rounds 3 > $OUT/c2.log 2>&1 || exit 1
tail -1 $OUT/c2.log
