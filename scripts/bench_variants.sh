# bench line of each library variant (default: the product build + listed variants)
#   VARIANTS="base w12" BENCH_ARGS="--rows 100000000" bash scripts/bench_variants.sh
# (variants that skip work fail verification: exit 3 is reported, not fatal)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-variants}
mkdir -p $OUT
for v in ${VARIANTS:-base}; do
  L=$PWD/cq_amd/lib/libcqgpu_$v.so
  [ $v = base ] && L=$PWD/cq_amd/lib/libcqgpu.so
  CQ_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-config2 --gen-workers 8 ${BENCH_ARGS:-} > $OUT/$v.json 2> $OUT/$v.err
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { tail -5 $OUT/$v.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$v.json')); r=d['roofline']; print('$v', round(r['kernel_ms'],3), 'ms', round(r['frac'],3), 'verified', d['verified'])"
done
if [ -n "$LDSPMC" ]; then
  B="python bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --no-config2 --gen-workers 8"
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv -d $OUT/lds -o run -- $B > $OUT/lds.log 2>&1 || exit 1

fi
