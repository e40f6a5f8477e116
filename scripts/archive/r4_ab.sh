# A/B of scan_kernel's MIN/MAX update (lib variants under cq_amd/lib/ab) plus
# the scan tests and a traced config-3 bench (GPU box):  TAG=x bash scripts/r4_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4ab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_groupby.py tests/test_gpu_lean.py tests/test_gpu_partials.py -m gpu -q -x --timeout 160 --timeout-method thread > $OUT/pt.log 2>&1
echo "pt rc=$?"; tail -2 $OUT/pt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-config5 > $OUT/kt.json 2> $OUT/kt.err || { echo kt failed; exit 1; }
timeout -k 10 200 python scripts/r4_other_kernels.py --steps 4 > $OUT/o_main.log 2>&1 || { echo main failed; tail -5 $OUT/o_main.log; exit 1; }
for v in NOSNAP SKIP; do
  CQ_AMD_LIB=cq_amd/lib/ab/libcqgpu_$v.so timeout -k 10 200 python scripts/r4_other_kernels.py --steps 4 > $OUT/o_$v.log 2>&1 || { echo $v failed; tail -5 $OUT/o_$v.log; exit 1; }
done
grep -h "^scan_kernel" $OUT/o_*.log
