# full GPU suite, then config 3 / 2 bench lines, the config-5 leg and a kernel trace
# of the config-3 step (GPU box):  TAG=x bash scripts/r4_round.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?"; tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --steps 30 > $OUT/bench3.json 2> $OUT/bench3.err || exit 1
timeout -k 10 200 python -u bench.py --config 2 --no-cpu --no-e2e --no-config5 --steps 30 > $OUT/bench2.json 2> $OUT/bench2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $OUT/kt.json 2> $OUT/kt.err || exit 1
echo done
