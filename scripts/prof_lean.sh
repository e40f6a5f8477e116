# lean_kernel stage variants + SQ counters of the full kernel (one GPU call)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-leanprof}
mkdir -p $OUT
VARIANTS="${VARIANTS:-l0 l1 l2 l3 base}" PROF_TAG=${PROF_TAG:-leanprof} bash scripts/prof_variants.sh || exit 1
B="python bench.py --steps 5 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $OUT/sq2 -o run -- $B > $OUT/sq2.log 2>&1 || { tail $OUT/sq2.log; exit 1; }
echo done
