# instruction mix of the scan kernel per profiling stage (10M rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-pmcst}
mkdir -p $OUT
B="python bench.py --rows 10000000 --steps 2 --warmup 1 --no-cpu"
for st in 1 2 3; do
  L=$PWD/cq_amd/lib/libcqgpu_s$st.so
  [ $st = 3 ] && L=$PWD/cq_amd/lib/libcqgpu.so
  CQ_AMD_LIB=$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/s$st -o run -- $B > $OUT/s$st.log 2>&1 || exit 1
done
