# lean_kernel stall diagnosis: SQ counter passes (8 SQ counters each) over the config-3 bench
#   LIB=cq_amd/lib/libcqgpu.so TAG=x bash scripts/r3_pmc.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3pmc}
mkdir -p $OUT
L=${LIB:-$PWD/cq_amd/lib/libcqgpu.so}
B="python bench.py --rows ${ROWS:-20000000} --steps 5 --warmup 1 --no-cpu --no-e2e --no-config2 --gen-workers 8"
i=0
for C in "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CU_CYCLES" \
         "SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_IFETCH SQ_INSTS_LDS_ATOMIC" \
         ${EXTRA_PASSES}; do
  i=$((i+1))
  CQ_AMD_LIB=$L timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o run -- $B > $OUT/p$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "pass $i rc=$rc"; tail -5 $OUT/p$i.log; exit 1; }
done
python - "$OUT" <<'PY'
import collections, csv, glob, json, sys
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "lean_kernel" in r["Kernel_Name"] or "fast_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
a = {c: sum(x.values()) / len(x) for c, x in tot.items()}
json.dump(a, open(f"{out}/pmc.json", "w"), indent=1)
for k in sorted(a): print(f"{k:28s} {a[k]:.4g}")
PY
