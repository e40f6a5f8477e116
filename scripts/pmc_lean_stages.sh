# instruction mix of lean_kernel per profiling stage (10M rows), one rocprofv3 pass each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-pmclean}
mkdir -p $OUT
B="python bench.py --rows 10000000 --steps 2 --warmup 1 --no-cpu --no-e2e --no-config2"
for st in ${STAGES:-l0 l1 l2 l3 base}; do
  L=$PWD/cq_amd/lib/libcqgpu_$st.so
  [ $st = base ] && L=$PWD/cq_amd/lib/libcqgpu.so
  CQ_AMD_LIB=$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/$st -o run -- $B > $OUT/$st.log 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit 1   # 3: a stage build fails verification by design
  [ -n "$NOBENCH" ] && continue
  CQ_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $OUT/$st.json 2> $OUT/$st.err || exit 1
  python -c "import json; d=json.load(open('$OUT/$st.json')); print('$st', round(d['roofline']['kernel_ms'],3), 'ms')"
done
