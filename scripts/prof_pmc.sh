# PMC passes over the bench's scan kernel (each counter group in its own run,
# kernel-trace/stats only beside --pmc, as the pool requires)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-pmc}
mkdir -p $OUT
ROWS=${ROWS:-10000000}
B="python bench.py --rows $ROWS --steps 3 --warmup 1 --no-cpu --no-e2e --no-config2 --gen-workers 8"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B > $OUT/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_SALU SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_SMEM --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_LDS_ATOMIC SQ_BUSY_CYCLES --output-format csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o run -- $B > $OUT/p3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/p4 -o run -- $B > $OUT/p4.log 2>&1
echo "rc=$?"
[ -n "$CLK" ] && CQ_AMD_LIB=$PWD/cq_amd/lib/libcqgpu_clk.so timeout -k 10 300 python scripts/lean_clocks.py > $OUT/clk.txt 2>&1; cat $OUT/clk.txt 2>/dev/null
