# round 6: the probe side's one-pass typed send (ROUTE 3) -- typed tests, then the
# config-5 rank step one-pass vs two-pass on the same box, and its kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6s
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_join_dist.py tests/test_gpu_dist_rccl.py -m gpu -x -q -k "typed or rccl" --timeout 200 --timeout-method thread > $OUT/pt.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $OUT/pt.log | tail -2
[ $rc -eq 0 ] || { tail -30 $OUT/pt.log; exit $rc; }
timeout -k 10 300 python scripts/r6_config5_profile.py > $OUT/one.json 2> $OUT/one.err || { tail -20 $OUT/one.err; exit 1; }
CQGPU_TYPED_TWO_PASS=1 timeout -k 10 300 python scripts/r6_config5_profile.py > $OUT/two.json 2> $OUT/two.err || { tail -20 $OUT/two.err; exit 1; }
timeout -k 10 300 python scripts/r6_config5_profile.py > $OUT/one_b.json 2> $OUT/one_b.err || exit 1
for f in one two one_b; do python -c "
import json; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1])
print('$f', round(d['step_s']*1e3,3), d['phases_ms'], d['verified'], d['recv_entries'], d['xgmi_sent_bytes'])
"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/r6_config5_profile.py --steps 3 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
echo "prof rc=$?"
