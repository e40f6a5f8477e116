# Time the scan kernel with parts of the per-record work compiled out
# (CQ_PROF_STAGE=1: split + classify only; 2: + field walk and typing).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-stages}
mkdir -p $OUT
for st in 1 2; do
  timeout -k 10 300 env CQ_AMD_LIB=$PWD/cq_amd/lib/libcqgpu_s$st.so python bench.py --steps 5 --warmup 1 --no-cpu > $OUT/s$st.json 2> $OUT/s$st.err || exit 1
done
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $OUT/s3.json 2> $OUT/s3.err || exit 1
for st in 1 2 3; do python -c "import json,sys; d=json.load(open('$OUT/s$st.json')); print('stage $st', d['roofline']['kernel_ms'], 'ms')"; done
