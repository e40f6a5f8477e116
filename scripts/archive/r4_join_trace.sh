# kernel trace of the config-5 join at full size (GPU box):  TAG=x bash scripts/r4_join_trace.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4jt}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/jt -o run -- python scripts/join_variant_bench.py base --steps 6 --rounds 1 > $OUT/jt.log 2>&1 || { echo jt failed; tail -5 $OUT/jt.log; exit 1; }
grep "scan_ms" $OUT/jt.log
