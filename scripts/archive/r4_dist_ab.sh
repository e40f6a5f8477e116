# Round 4: the N > 1 step at world size 1 over RCCL (CQ_BENCH_FORCE_DIST), the
# library-side merge (default) against round 3's Python-driven dense merge
# (CQ_BENCH_DIST_PY=1), same box, 1e8 rows of config 3's file.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r4dist}
mkdir -p $OUT
run() {   # $1 = label, rest = env
  local label=$1; shift
  env "$@" CQ_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
      --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 1 --steps 20 --warmup 3 \
      --rows ${ROWS:-100000000} --no-cpu --no-e2e --no-config2 --no-config5 > $OUT/$label.json 2> $OUT/$label.err
}
run lib && run py CQ_BENCH_DIST_PY=1 && run lib2 || exit $?
for f in lib py lib2; do python - "$OUT/$f.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], "ms_per_step %.3f kernel_ms %.3f overhead %.3f verified %s %s" % (
    d["ms_per_step"], d["roofline"]["kernel_ms"], d["ms_per_step"] - d["roofline"]["kernel_ms"], d["verified"],
    d["config"]["parallelism"]))
PY
done
