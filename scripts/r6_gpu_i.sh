# round 6: config-5 rank step under rocprofv3 (kernel stats + phase timing)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6i
mkdir -p $OUT
CQ_AMD_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c5 -- python scripts/r6_config5_profile.py --steps 3 > $OUT/c5.txt 2> $OUT/c5.err
echo "prof rc=$?"; tail -1 $OUT/c5.txt | cut -c1-600; grep "cq_amd timing" $OUT/c5.err | tail -30
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -30
