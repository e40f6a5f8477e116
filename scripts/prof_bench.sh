set -o pipefail
mkdir -p gpurun_out/prof1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/prof1/counters.txt 2>&1 || true
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-rows 2000000 > gpurun_out/prof1/bench.json 2> gpurun_out/prof1/bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1/kt -o run -- python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof1/kt.log 2>&1
echo done
