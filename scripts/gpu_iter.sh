# one iteration on the GPU: lean parity, the whole GPU suite, a bench line and one
# PMC pass of the scan kernel (10M rows).  SKIP_ALL=1 skips the whole suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-iter}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lean.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_lean.log 2>&1
rc=$?; tail -15 $OUT/pytest_lean.log; [ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_ALL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_all.log 2>&1
  rc=$?; tail -5 $OUT/pytest_all.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/base -o run -- python bench.py --rows 10000000 --steps 2 --warmup 1 --no-cpu > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
echo done
if [ -f cq_amd/lib/libcqgpu_clk.so ]; then
  CQ_AMD_LIB=$PWD/cq_amd/lib/libcqgpu_clk.so timeout -k 10 300 python scripts/lean_clocks.py 20000000 > $OUT/clocks.txt 2>&1 || { tail $OUT/clocks.txt; exit 1; }
  cat $OUT/clocks.txt
fi
