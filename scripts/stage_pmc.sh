# per-stage profile of lean_kernel: for each library variant (stage builds from
# build_lean_variants.sh, "base" = the product build) the kernel time at ROWS rows
# and one PMC pass of SQ counters.  TAG=x VARIANTS="p1 p2 base" bash scripts/stage_pmc.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-stages}
mkdir -p $OUT
ROWS=${ROWS:-20000000}
CTRS=${CTRS:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"}
for v in ${VARIANTS:-base}; do
  L=$PWD/cq_amd/lib/libcqgpu_$v.so
  [ $v = base ] && L=$PWD/cq_amd/lib/libcqgpu.so
  B="python bench.py --rows $ROWS --steps 5 --warmup 1 --no-cpu --no-e2e --no-config2 --gen-workers 8"
  CQ_AMD_LIB=$L timeout -k 10 300 $B > $OUT/$v.json 2> $OUT/$v.err
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { tail -5 $OUT/$v.err; exit 1; }
  CQ_AMD_LIB=$L timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/pmc_$v -o run -- $B > $OUT/pmc_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { tail -5 $OUT/pmc_$v.log; exit 1; }
  python - "$OUT" "$v" <<'PY'
import collections, csv, glob, json, sys
out, v = sys.argv[1], sys.argv[2]
d = json.load(open(f"{out}/{v}.json"))
nb = d["config"]["bytes_per_gpu"]; wins = nb / 3968.0
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{out}/pmc_{v}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "lean_kernel" in r["Kernel_Name"] or "fast_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
a = {c: sum(x.values()) / len(x) / wins for c, x in tot.items()}
wc = a.get("SQ_WAVE_CYCLES", 1)
print(f"{v:6s} {d['roofline']['kernel_ms']:.3f} ms | per 3968B: VALU {a.get('SQ_INSTS_VALU',0):.0f} SALU {a.get('SQ_INSTS_SALU',0):.0f} "
      f"LDS {a.get('SQ_INSTS_LDS',0):.1f} bankconf {a.get('SQ_LDS_BANK_CONFLICT',0):.0f} | wait {a.get('SQ_WAIT_ANY',0)/wc:.2f} "
      f"waitinst {a.get('SQ_WAIT_INST_ANY',0)/wc:.2f} active {a.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} wavecyc {wc:.0f}")
PY
done
