# time every profiling build of the scan kernel (bench workload, 100M rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-variants}
mkdir -p $OUT
for v in ${VARIANTS:-s0 s0p s1 s1n s2 s3p base}; do
  L=$PWD/cq_amd/lib/libcqgpu_$v.so
  [ $v = base ] && L=$PWD/cq_amd/lib/libcqgpu.so
  CQ_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $OUT/$v.json 2> $OUT/$v.err || exit 1
  python -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', round(d['roofline']['kernel_ms'],3), 'ms')"
done
