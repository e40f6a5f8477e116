# profiling builds of libcqgpu.so with lean.hip compiled to stop after a stage
# (LEAN_PROF=0 loads+staging, 1 +classify/numbering, 2 +field walk, 3 +values/keys)
set -e
cd "$(dirname "$0")/../cq_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include"
for v in ${STAGES:-0 1 2 3}; do
  ( hipcc $F -DLEAN_PROF=$v -c lean.hip -o /tmp/lean_l$v.o && \
    hipcc -shared --offload-arch=gfx950 -o ../lib/libcqgpu_l$v.so ../lib/scan.o /tmp/lean_l$v.o ../lib/executor.o ../lib/sort.o ) &
done
wait
