# three-record pass (ungrouped, short records) A/B on config 2 and the fast-path GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rp}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_partials.py tests/test_gpu_lean.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="python bench.py --config 2 --steps 20 --warmup 3 --no-cpu --no-e2e --no-config5 --gen-workers 8"
for i in 1 2; do
  timeout -k 10 200 $B > $OUT/rp3_$i.json 2> $OUT/rp3.err || exit 1
  CQGPU_FAST_RP2=1 timeout -k 10 200 $B > $OUT/rp2_$i.json 2> $OUT/rp2.err || exit 1
done
for f in rp3_1 rp2_1 rp3_2 rp2_2; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), d['verified'])"; done
