# kernel time of library variants (cq_amd/lib/libcqgpu_<v>.so; "base" = the product
# build) on the config-3 bench, interleaved A/B rounds in separate processes:
#   VARIANTS="base a0 nl" ROUNDS=2 ROWS=100000000 bash scripts/variant_times.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-variants}
mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    L=$PWD/cq_amd/lib/libcqgpu_$v.so
    [ $v = base ] && L=$PWD/cq_amd/lib/libcqgpu.so
    CQ_AMD_LIB=$L timeout -k 10 240 python bench.py --rows ${ROWS:-100000000} --steps 10 --warmup 2 --no-cpu --no-e2e \
        --no-config2 --gen-workers 8 > $OUT/$v.$r.json 2> $OUT/$v.$r.err
    rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "$v rc=$rc"; tail -3 $OUT/$v.$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/$v.$r.json')); print('%-6s round $r kernel %.3f ms step %.3f ms verified %s' % ('$v', d['roofline']['kernel_ms'], d['ms_per_step'], d['verified']))"
  done
done
