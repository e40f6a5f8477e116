# one short bench line + PMC instruction mix of the scan kernel (10M rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-quick}
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_SALU SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR --output-format csv -d $OUT/p1 -o run -- python bench.py --rows 10000000 --steps 3 --warmup 1 --no-cpu > $OUT/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_LDS_ATOMIC SQ_BUSY_CYCLES --output-format csv -d $OUT/p2 -o run -- python bench.py --rows 10000000 --steps 3 --warmup 1 --no-cpu > $OUT/p2.log 2>&1
rc=$?
cat $OUT/bench.json
exit $rc
