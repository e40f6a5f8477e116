# lean parity + a bench line + the lean kernel's instruction counts (PMC, 10 M rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-it}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_lean.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --kernel-include-regex lean_kernel --output-format csv -d $OUT/pmc -o run -- python bench.py --rows 10000000 --steps 2 --warmup 1 --no-cpu > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
python scripts/pmc_lean_table.py $OUT/pmc 2>/dev/null || find $OUT/pmc -name '*counter_collection.csv' | head -1 | xargs -I{} python -c "
import csv,collections,sys
d=collections.defaultdict(list)
for r in csv.DictReader(open('{}')):
    if 'lean_kernel' in r['Kernel_Name']: d[r['Counter_Name']].append(float(r['Counter_Value']))
for k,v in d.items(): print(k, sum(v)/len(v))
"
