# round 6: typed receive build with the next key by DPP -- typed tests, config-5 step, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6v
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_join_dist.py -m gpu -x -q -k "typed" --timeout 200 --timeout-method thread > $OUT/pt.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $OUT/pt.log | tail -2
[ $rc -eq 0 ] || { tail -30 $OUT/pt.log; exit $rc; }
timeout -k 10 300 python scripts/r6_config5_profile.py --steps 10 > $OUT/c5b.json 2> $OUT/c5b.err || exit 1
python -c "
import json
for f in ('c5b',):
    d=json.loads(open('$OUT/'+f+'.json').read().strip().splitlines()[-1]); print(f, round(d['step_s']*1e3,3), d['phases_ms'], d['verified'])
"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o c5 -- python3 $GRAFT_REPO_ROOT/scripts/r6_config5_profile.py --steps 3 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
echo "prof rc=$?"
grep -E "jx_ent_build|jx_extract" $GRAFT_REPO_ROOT/$OUT/prof/c5_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
cd /tmp && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$OUT/fetch -o run -- python3 $GRAFT_REPO_ROOT/scripts/r6_config5_profile.py --steps 2 > $GRAFT_REPO_ROOT/$OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$OUT/write -o run -- python3 $GRAFT_REPO_ROOT/scripts/r6_config5_profile.py --steps 2 > $GRAFT_REPO_ROOT/$OUT/write.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python scripts/r6_config5_traffic.py $OUT $OUT/config5_traffic.json | head -14
