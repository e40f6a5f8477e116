# HIP API + kernel trace summary of a short bench run (host overhead per query)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-api}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --stats --output-format csv -d $OUT/rt -o run -- python bench.py --rows 20000000 --steps 20 --warmup 2 --no-cpu > $OUT/rt.log 2>&1 || { tail $OUT/rt.log; exit 1; }
ls $OUT/rt
