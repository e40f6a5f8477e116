# untraced bench (the driver's view) then a traced one for the step timeline,
# then the scan tests (GPU box):  TAG=x bash scripts/r4_bench_pair.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4bp}
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -5 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-config5 > $OUT/kt.json 2> $OUT/kt.err || { echo kt failed; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_groupby.py tests/test_gpu_lean.py tests/test_gpu_partials.py -m gpu -v -x --timeout 160 --timeout-method thread > $OUT/pt.log 2>&1
echo "pt rc=$?"; tail -2 $OUT/pt.log
