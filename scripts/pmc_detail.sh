# stall/issue counters of the scan kernel (10M rows) per build variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-pmcd}
rm -rf $OUT; mkdir -p $OUT
B="python bench.py --rows 10000000 --steps 2 --warmup 1 --no-cpu"
for v in ${VARIANTS:-s1 s2 base}; do
  L=$PWD/cq_amd/lib/libcqgpu_$v.so
  [ $v = base ] && L=$PWD/cq_amd/lib/libcqgpu.so
  CQ_AMD_LIB=$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $OUT/${v}_a -o run -- $B > $OUT/${v}_a.log 2>&1 || exit 1
  CQ_AMD_LIB=$L timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES --output-format csv -d $OUT/${v}_b -o run -- $B > $OUT/${v}_b.log 2>&1 || exit 1
done
