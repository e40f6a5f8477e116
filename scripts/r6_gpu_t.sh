# round 6: typed receive build (next key by lane shuffle) + merge scratch reuse --
# join tests, the config-5 rank step, its kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6u
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_join_dist.py tests/test_gpu_dist_rccl.py -m gpu -x -q -k "typed or rccl" --timeout 200 --timeout-method thread > $OUT/pt.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $OUT/pt.log | tail -2
[ $rc -eq 0 ] || { tail -30 $OUT/pt.log; exit $rc; }
CQ_AMD_TIMING=1 timeout -k 10 300 python scripts/r6_config5_profile.py --steps 10 > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
timeout -k 10 300 python scripts/r6_config5_profile.py --steps 10 > $OUT/c5b.json 2> $OUT/c5b.err || exit 1
python -c "
import json
for f in ('c5','c5b'):
    d=json.loads(open('$OUT/'+f+'.json').read().strip().splitlines()[-1]); print(f, round(d['step_s']*1e3,3), d['phases_ms'], d['verified'])
"
grep "merge" $OUT/c5.err | tail -3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o c5 -- python3 $GRAFT_REPO_ROOT/scripts/r6_config5_profile.py --steps 3 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
echo "prof rc=$?"
