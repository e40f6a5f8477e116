# round 6: replicated routing (mixed key classes, JOIN without ON across partials), then
# the whole GPU suite, smoke and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6h
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_join_dist.py -m gpu -x -q --timeout 200 \
   --timeout-method thread -k "typed" > $OUT/pt_x.log 2>&1
rc=$?; echo "targeted rc=$rc"; tail -25 $OUT/pt_x.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pt.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -15 $OUT/pt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python __graft_entry__.py smoke > $OUT/smoke.txt 2>&1 || exit 1
tail -1 $OUT/smoke.txt
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','ms_per_step')}, d['roofline'])
c5=d.get('config5') or {}; print('config5', {k: c5.get(k) for k in ('value','ms_per_step','phases_ms','verified','exchange')}, (c5.get('roofline') or {}).get('frac'))
print('e2e', d.get('end_to_end')); print('cpu', d.get('cpu_baseline'))
"
tail -3 $OUT/bench.err
