# round 6: compound WHERE leaves evaluated once per pass -- fast-kernel tests, the other
# plan shapes' rooflines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6m
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pt.log 2>&1
rc=$?; echo "fast rc=$rc"; tail -2 $OUT/pt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/r6_other_kernels.py > $OUT/other.txt 2> $OUT/other.err || { tail -5 $OUT/other.err; exit 1; }
python -c "
import json
for l in open('$OUT/other.txt'):
    if l.startswith('{'):
        for k,v in json.loads(l)['results'].items(): print(f\"{k:60s} {v.get('kernel')} {v.get('kernel_ms')} {v.get('frac')}\")
"
