# round 6 (re-entry): the whole GPU suite at HEAD, smoke, and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6r
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --durations=25 > $OUT/pt.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" $OUT/pt.log | tail -2
[ $rc -eq 0 ] || { tail -30 $OUT/pt.log; exit $rc; }
timeout -k 10 120 python __graft_entry__.py smoke > $OUT/smoke.txt 2>&1 || exit 1
tail -1 $OUT/smoke.txt
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','ms_per_step')}, d['roofline']['frac'], d['roofline']['kernel_ms'])
c5=d.get('config5') or {}; print('config5', c5.get('ms_per_step'), c5.get('phases_ms'), c5.get('verified'))
print('config2', d['config2']['roofline_frac'], 'e2e', d.get('end_to_end',{}).get('GB_per_s'))
"
