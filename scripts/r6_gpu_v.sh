# round 6 (re-entry, final tree): config-5 HBM traffic passes, the whole GPU suite,
# smoke and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6w
mkdir -p $OUT
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$OUT/fetch -o run -- python3 $R/scripts/r6_config5_profile.py --steps 2 > $R/$OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$OUT/write -o run -- python3 $R/scripts/r6_config5_profile.py --steps 2 > $R/$OUT/write.log 2>&1 || exit 1
cd $R && python scripts/r6_config5_traffic.py $OUT $OUT/config5_traffic.json > $OUT/traffic.txt && head -3 $OUT/traffic.txt
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --durations=10 > $OUT/pt.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" $OUT/pt.log | tail -2
[ $rc -eq 0 ] || { tail -30 $OUT/pt.log; exit $rc; }
timeout -k 10 120 python __graft_entry__.py smoke > $OUT/smoke.txt 2>&1 || exit 1
tail -1 $OUT/smoke.txt
cp $OUT/config5_traffic.json profiles/config5_traffic.json
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','ms_per_step')}, d['roofline']['frac'], d['roofline']['kernel_ms'])
c5=d.get('config5') or {}; print('config5', c5.get('ms_per_step'), c5.get('phases_ms'), c5.get('verified'), c5.get('roofline',{}).get('frac'))
print('config2', d['config2']['roofline_frac'], 'e2e', d.get('end_to_end',{}).get('GB_per_s'))
"
