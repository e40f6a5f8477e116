# round 6: streamed blob merge + continuous upload pipeline -- the whole GPU suite, then
# the end-to-end ingest over chunk sizes / threads, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6k
mkdir -p $OUT
timeout -k 10 750 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pt.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -4 $OUT/pt.log
[ $rc -eq 0 ] || exit $rc
for cfg in "8 16" "8 8" "16 16" "12 32" "8 32"; do
  set -- $cfg
  CQGPU_UPLOAD_THREADS=$1 CQGPU_UPLOAD_CHUNK_MB=$2 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --no-config2 --no-config5 > $OUT/e2e_$1_$2.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$OUT/e2e_$1_$2.json').read().strip().splitlines()[-1]); e=d['end_to_end']; print('threads $1 chunk $2 MB:', round(e['GB_per_s'],1), 'GB/s', e['verified'])"
done
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','ms_per_step')}, d['roofline']['frac'])
c5=d.get('config5') or {}; print('config5', c5.get('ms_per_step'), c5.get('phases_ms'), c5.get('verified'))
print('e2e', d.get('end_to_end',{}).get('GB_per_s'))
"
