# round 6: compound WHERE (LDS leaves), typed exchange tests, rooflines, bench (config 5 whole rank step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pt_fast.log 2>&1
echo "fast rc=$?"; tail -3 $OUT/pt_fast.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_join_dist.py -m gpu -x -q --timeout 200 --timeout-method thread -k "typed or first_ids or projection_bytes" > $OUT/pt_typed.log 2>&1
echo "typed rc=$?"; tail -15 $OUT/pt_typed.log
timeout -k 10 400 python scripts/r6_other_kernels.py > $OUT/other.txt 2>&1; echo "other rc=$?"; grep -v "^{" $OUT/other.txt | cut -c1-60,150-330
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','ms_per_step')}, d['roofline']['frac'])
c5=d.get('config5') or {}; print('config5', {k: c5.get(k) for k in ('value','ms_per_step','phases_ms','verified','exchange')}, (c5.get('roofline') or {}).get('frac'))
print('e2e', d.get('end_to_end'))
"
tail -3 $OUT/bench.err
