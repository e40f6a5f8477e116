# round 6: the typed receive's rising-keys form -- typed tests, the config-5 rank step
# and the end-to-end ingest sweep repeated (threads x chunk MB)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6n
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_join_dist.py -m gpu -x -q --timeout 200 --timeout-method thread \
   -k "typed" > $OUT/pt.log 2>&1
rc=$?; echo "typed rc=$rc"; tail -2 $OUT/pt.log
[ $rc -eq 0 ] || exit $rc
CQ_AMD_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c5 -- python scripts/r6_config5_profile.py --steps 5 > $OUT/c5.txt 2> $OUT/c5.err
echo "prof rc=$?"; tail -1 $OUT/c5.txt | cut -c1-330
for rep in; do
for cfg in "8 32" "16 32" "8 64" "12 16"; do
  set -- $cfg
  CQGPU_UPLOAD_THREADS=$1 CQGPU_UPLOAD_CHUNK_MB=$2 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --no-config2 --no-config5 > $OUT/e2e.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$OUT/e2e.json').read().strip().splitlines()[-1]); e=d['end_to_end']; print('rep $rep threads $1 chunk $2 MB:', round(e['GB_per_s'],1), 'GB/s', round(e['seconds']*1e3,1), 'ms', e['verified'])" | tee -a $OUT/ingest.txt
done
done
