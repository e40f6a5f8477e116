# per-phase clocks + stage-variant timings of the scan kernel (one GPU call)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-phase}
mkdir -p $OUT
CQ_AMD_LIB=$PWD/cq_amd/lib/libcqgpu_clk.so timeout -k 10 300 python scripts/clocks.py 20000000 > $OUT/clocks.txt 2>&1 || { cat $OUT/clocks.txt; exit 1; }
cat $OUT/clocks.txt
VARIANTS="${VARIANTS:-s0 s1 s1n noins base}" bash scripts/prof_variants.sh
