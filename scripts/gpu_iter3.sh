# parity (lean + general), config-3 and config-2 bench lines, lean instruction counts
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-it}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_lean.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --config 2 --steps 10 --warmup 2 --no-cpu > $OUT/bench2.json 2> $OUT/bench2.err || { tail $OUT/bench2.err; exit 1; }
python - <<'PY'
import json,os
o=os.environ.get("TAG","it")
for f in ("bench.json","bench2.json"):
    d=json.load(open(f"gpurun_out/{o}/{f}"))
    print(f, d["config"]["workload"][:8], "kernel_ms %.3f" % d["roofline"]["kernel_ms"], "frac %.3f" % d["roofline"]["frac"], "rows/s %.3g" % d["value"])
PY
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --kernel-include-regex lean_kernel --output-format csv -d $OUT/pmc -o run -- python bench.py --rows 10000000 --steps 2 --warmup 1 --no-cpu > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
