# fast_kernel variants, host phase times and a short kernel trace of the bench step
#   TAG=x VARIANTS="base onk" bash scripts/r3_overhead.sh   (on the GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ovh}
mkdir -p $OUT
timeout -k 10 420 python -u scripts/variant_bench.py ${VARIANTS:-base} --rounds 3 --steps 10 > $OUT/c3.log 2>&1 || exit 1
tail -1 $OUT/c3.log
CQ_AMD_TIMING=1 timeout -k 10 200 python -u scripts/host_overhead.py 20000000 > $OUT/host.log 2>&1 || exit 1
tail -12 $OUT/host.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-config5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json
