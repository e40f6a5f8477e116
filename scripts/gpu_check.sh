# parity tests through the C ABI, then one short bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/check
timeout -k 10 600 python -m pytest tests/test_gpu_tokenizer.py tests/test_gpu_parity.py tests/test_gpu_rows.py -m gpu -x -q \
    --timeout 120 > gpurun_out/check/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/check/bench.json 2> gpurun_out/check/bench.err
rc=$?
tail -5 gpurun_out/check/pytest.log
cat gpurun_out/check/bench.json
exit $rc
