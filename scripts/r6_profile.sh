# round 6 evidence: the other plan shapes' rooflines, then rocprofv3 over one bench
# process (configs 3, 2 and 5): kernel trace + stats, HBM traffic and SQ counter passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6p
mkdir -p $OUT
timeout -k 10 300 python scripts/r6_other_kernels.py > $OUT/other.txt 2> $OUT/other.err || { tail -5 $OUT/other.err; exit 1; }
grep -v '^{' $OUT/other.txt | cut -c1-150
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --gen-workers 8"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B > $OUT/kt.log 2>&1 || exit 1
echo kt done
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit 1
echo traffic done
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 || exit 1
echo done
