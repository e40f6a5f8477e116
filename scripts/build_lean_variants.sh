# profiling builds of libcqgpu.so with lean.hip compiled to stop after a stage
# (LEAN_PROF=0 loads+staging, 1 +classify/numbering, 2 +field walk and loads,
# 3 +values/keys) or with no HBM reads after the first window (nomem)
set -e
cd "$(dirname "$0")/../cq_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include"
for v in ${VARIANTS:-"l0:-DLEAN_PROF=0" "l1:-DLEAN_PROF=1" "l2:-DLEAN_PROF=2" "l3:-DLEAN_PROF=3" "nomem:-DLEAN_NOMEM"}; do
  n=${v%%:*}; d=${v#*:}
  ( hipcc $F $d -c lean.hip -o /tmp/lean_$n.o 2>/dev/null && \
    hipcc -shared --offload-arch=gfx950 -o ../lib/libcqgpu_$n.so ../lib/scan.o /tmp/lean_$n.o ../lib/executor.o ../lib/sort.o ../lib/hostcell.o ) &
done
wait
