# round 6: compound WHERE on fast_kernel, multi-rank host backend, other-kernel rooflines, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_dist_rccl.py tests/test_gpu_join_dist.py -m gpu -x -v \
   --timeout 200 --timeout-method thread -k "fast or host_backend or failure_reaches or projection_bytes or first_ids" > $OUT/pt.log 2>&1
rc=$?; tail -15 $OUT/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/r6_other_kernels.py > $OUT/other.txt 2>&1; rc=$?; cat $OUT/other.txt | grep -v "^{" ; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/bench.json 2> $OUT/bench.err; rc=$?
cat $OUT/bench.json; tail -3 $OUT/bench.err; exit $rc
