# round 6: config-5 rank step's host phases (CQ_AMD_TIMING=1) after the one-pass probe send
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6t
mkdir -p $OUT
CQ_AMD_TIMING=1 timeout -k 10 300 python scripts/r6_config5_profile.py --steps 3 > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
timeout -k 10 300 python scripts/r6_config5_profile.py --steps 10 > $OUT/c5b.json 2> $OUT/c5b.err || exit 1
python -c "
import json
for f in ('c5','c5b'):
    d=json.loads(open('$OUT/'+f+'.json').read().strip().splitlines()[-1]); print(f, round(d['step_s']*1e3,3), d['phases_ms'], d['verified'])
"
grep "timing" $OUT/c5.err | tail -40
