# round-3 first look: counter list, baseline bench (config 3 at 1e8 rows), and a
# PC-sampling attempt on lean_kernel (stochastic, then host_trap)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r3probe
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "list failed rc=$?"
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --gen-workers 8"
timeout -k 10 300 $B > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
B2="python bench.py --rows 20000000 --steps 3 --warmup 1 --no-cpu --no-e2e --no-config2 --gen-workers 8"
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
   --pc-sampling-interval 65536 --output-format csv -d $OUT/pcs -o run -- $B2 > $OUT/pcs.log 2>&1
echo "stochastic rc=$?"
tail -5 $OUT/pcs.log
ls -R $OUT/pcs | head -20
