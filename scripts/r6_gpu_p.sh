# round 6: typed-exchange tests and the config-5 rank step after a host-side change
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6q
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_join_dist.py tests/test_gpu_dist_rccl.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pt.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $OUT/pt.log | tail -2
[ $rc -eq 0 ] || { tail -30 $OUT/pt.log; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu --no-e2e > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','ms_per_step')}, d['roofline']['frac'])
c5=d.get('config5') or {}; print('config5', c5.get('ms_per_step'), c5.get('phases_ms'), c5.get('verified'))
"
