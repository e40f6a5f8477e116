# round 6: multi-rank host-backend tests + ingest A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6a
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_dist_rccl.py tests/test_gpu_join_dist.py -m gpu -x -v --timeout 150 --timeout-method thread \
   -k "host_backend or failure_reaches or one_rank or projection_bytes or first_ids" > $OUT/pt.log 2>&1
rc=$?; tail -30 $OUT/pt.log
head -c 3889108980 /dev/zero > /tmp/f.bin
timeout -k 10 200 ./scripts/micro/ingest /tmp/f.bin all 8 32 > $OUT/ingest.txt 2>&1
cat $OUT/ingest.txt
timeout -k 10 100 ./scripts/micro/ingest /tmp/f.bin pread 16 32 >> $OUT/ingest.txt 2>&1
timeout -k 10 100 ./scripts/micro/ingest /tmp/f.bin pread 8 64 >> $OUT/ingest.txt 2>&1
tail -6 $OUT/ingest.txt
timeout -k 10 300 python scripts/variant_bench.py base nob f3 --rounds 2 > $OUT/variants.txt 2>&1
cat $OUT/variants.txt
exit $rc
