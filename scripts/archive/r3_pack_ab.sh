# packed-result A/B (HBM pack + coalesced mailbox copy vs mapped writes) and GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pack}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_groupby.py tests/test_gpu_partials.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
B="python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-config5 --no-config2"
CQGPU_PACK_MAPPED=1 timeout -k 10 200 $B > $OUT/mapped.json 2>$OUT/mapped.err || exit 1
timeout -k 10 200 $B > $OUT/hbm.json 2>$OUT/hbm.err || exit 1
CQGPU_PACK_MAPPED=1 timeout -k 10 200 $B > $OUT/mapped2.json 2>>$OUT/mapped.err || exit 1
timeout -k 10 200 $B > $OUT/hbm2.json 2>>$OUT/hbm.err || exit 1
for f in mapped hbm mapped2 hbm2; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['verified'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt -o run -- $B > $OUT/kt.json 2> $OUT/kt.err || exit 1
python scripts/kt_timeline.py $OUT/kt/run_results.db | tail -12
