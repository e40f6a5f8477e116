# round 6: compound WHERE, typed join exchange (simulated ranks + host-backend ranks), rooflines, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6c
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py -m gpu -x -q --timeout 200 --timeout-method thread -k "compound" > $OUT/pt_fast.log 2>&1
echo "fast rc=$?"; tail -5 $OUT/pt_fast.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_join_dist.py -m gpu -x -q --timeout 200 --timeout-method thread -k "typed or first_ids or projection_bytes" > $OUT/pt_typed.log 2>&1
echo "typed rc=$?"; tail -25 $OUT/pt_typed.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_dist_rccl.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pt_dist.log 2>&1
echo "dist rc=$?"; tail -25 $OUT/pt_dist.log
timeout -k 10 400 python scripts/r6_other_kernels.py > $OUT/other.txt 2>&1; echo "other rc=$?"; grep -v "^{" $OUT/other.txt
