# config-5 join kernels: SQ / TCC counter passes over the bench's config-5 leg
#   TAG=x bash scripts/r4_join_pmc.sh     (GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4jpmc}
mkdir -p $OUT
B="python bench.py --rows 2000000 --steps 3 --warmup 1 --no-cpu --no-e2e --no-config2 --gen-workers 8"
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
         "FETCH_SIZE" "WRITE_SIZE SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" ; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o run -- $B > $OUT/p$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $i rc=$rc"; tail -5 $OUT/p$i.log; exit 1; }
done
python - "$OUT" <<'PY'
import collections, csv, glob, json, sys
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "jx_" not in n:
            continue
        k = n.split("(")[0][-60:]
        tot[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
res = {k: {c: sum(x.values()) / len(x) for c, x in cs.items()} for k, cs in tot.items()}
json.dump(res, open(f"{out}/pmc.json", "w"), indent=1)
for k, cs in res.items():
    print(k)
    for c in sorted(cs):
        print(f"   {c:28s} {cs[c]:.4g}")
PY
