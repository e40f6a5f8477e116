# round 6: partitioned probe over typed entries -- tests, then the config-5 rank step profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6j
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_join_dist.py -m gpu -x -q --timeout 200 --timeout-method thread \
   -k "typed" > $OUT/pt.log 2>&1
rc=$?; echo "typed rc=$rc"; tail -4 $OUT/pt.log
[ $rc -eq 0 ] || exit $rc
CQ_AMD_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c5 -- python scripts/r6_config5_profile.py --steps 3 > $OUT/c5.txt 2> $OUT/c5.err
echo "prof rc=$?"; tail -1 $OUT/c5.txt | cut -c1-400; grep "cq_amd timing" $OUT/c5.err | tail -4
