# Round-end evidence: GPU tests, the default bench line, and rocprofv3 summaries of
# the same bench command (kernel trace + HBM traffic PMC passes).
#   PROF_TAG=r3 bash scripts/round_profile.sh      (writes gpurun_out/$PROF_TAG)
#   NOTESTS=1 / NOBENCH=1 skip the test suite / the full bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-r3}
mkdir -p $OUT
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
# one process holds config 3 (fast_kernel<true,...>), config 2 (fast_kernel<false,...>)
# and config 5 (jx_* kernels): the summaries split the counters by kernel name
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --gen-workers 8"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B > $OUT/kt.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM --output-format csv -d $OUT/sq2 -o run -- $B > $OUT/sq2.log 2>&1 || exit 1
echo done
