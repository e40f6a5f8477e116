# the scan tests, a traced config-3 bench and the other
# scans' roofline with their kernel trace (GPU box):  TAG=x bash scripts/r4_batch.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4b}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_groupby.py tests/test_gpu_lean.py tests/test_gpu_partials.py -m gpu -v -x --timeout 160 --timeout-method thread > $OUT/pt.log 2>&1
echo "pt rc=$?"; tail -2 $OUT/pt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-config5 > $OUT/kt.json 2> $OUT/kt.err || { echo kt failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/ok -o run -- python scripts/r4_other_kernels.py > $OUT/other.log 2>&1 || { echo other failed; tail -5 $OUT/other.log; exit 1; }
tail -4 $OUT/other.log
CQ_AMD_TIMING=1 timeout -k 10 200 python scripts/r4_host_phases.py > $OUT/host.log 2> $OUT/host.err || { echo host failed; tail -5 $OUT/host.err; exit 1; }
cat $OUT/host.log; tail -3 $OUT/host.err
