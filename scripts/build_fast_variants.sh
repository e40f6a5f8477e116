# profiling builds of libcqgpu.so with fast.hip compiled differently (stage cut-offs):
#   VARIANTS="f1:-DFAST_PROF=1 f2:-DFAST_PROF=2 f3:-DFAST_PROF=3" bash scripts/build_fast_variants.sh
# (FAST_PROF=1: load + classify + record starts; =2: + views and the field walk;
#  =3: + field loads, typing, keys, hashes; the results of these builds are wrong)
set -e
cd "$(dirname "$0")/../cq_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include -mllvm -amdgpu-sched-strategy=max-ilp"
for v in ${VARIANTS:-"f1:-DFAST_PROF=1" "f2:-DFAST_PROF=2" "f3:-DFAST_PROF=3"}; do
  n=${v%%:*}; d=$(echo "${v#*:}" | tr "+" " ")
  ( /opt/rocm/bin/hipcc $F $d -c fast.hip -o /tmp/fast_$n.o && \
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib/libcqgpu_$n.so ../lib/scan.o ../lib/lean.o /tmp/fast_$n.o \
        ../lib/executor.o ../lib/route.o ../lib/prim.o ../lib/writer.o ../lib/merge.o ../lib/hostcell.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib ) &
done
wait
