# round 6: typed exchange tests + config 5 rank-step profile (phases + kernel trace)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6e
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_join_dist.py -m gpu -x -q --timeout 200 --timeout-method thread -k "typed or first_ids or projection_bytes" > $OUT/pt_typed.log 2>&1
echo "typed rc=$?"; tail -3 $OUT/pt_typed.log
CQ_AMD_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c5 -- python scripts/r6_config5_profile.py --steps 3 > $OUT/c5.txt 2> $OUT/c5.err
echo "prof rc=$?"; tail -2 $OUT/c5.txt | cut -c1-800; grep "cq_amd timing" $OUT/c5.err | tail -12
find $OUT/prof -name "*kernel_stats.csv" | head -3
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -25
