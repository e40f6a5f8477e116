# join tests, the config-5 scan time with host phases, and a kernel trace (GPU box):
#   TAG=x bash scripts/r4_join_check.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4jc}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fastjoin.py tests/test_gpu_join.py -m gpu -v -x --timeout 120 --timeout-method thread > $OUT/pt.log 2>&1
rc=$?; echo "pt rc=$rc"; tail -1 $OUT/pt.log; [ $rc -eq 0 ] || exit 1
CQ_AMD_TIMING=1 timeout -k 10 150 python scripts/join_variant_bench.py base --steps 6 --rounds 1 > $OUT/jt.log 2>&1 || { echo jt failed; tail -5 $OUT/jt.log; exit 1; }
tail -3 $OUT/jt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o run -- python scripts/join_variant_bench.py base --steps 6 --rounds 1 > $OUT/tr.log 2>&1 || { echo tr failed; tail -5 $OUT/tr.log; exit 1; }
echo done
