# profiling builds of libcqgpu.so with lean.hip compiled differently:
#   VARIANTS="clk:-DLEAN_CLK l1:-DLEAN_PROF=1 w12:-DLEAN_WAVES=12+-DLEAN_CLK" bash scripts/build_lean_variants.sh
# ("+" separates the flags of one variant)
# (LEAN_CLK: per-phase shader cycles; LEAN_PROF=1 stops after classify + record
# numbering; LEAN_NOMEM: no HBM reads after the first window)
set -e
cd "$(dirname "$0")/../cq_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-bitwise-instead-of-logical -I../../include"
for v in ${VARIANTS:-"clk:-DLEAN_CLK" "l1:-DLEAN_PROF=1" "nomem:-DLEAN_NOMEM"}; do
  n=${v%%:*}; d=$(echo "${v#*:}" | tr "+" " ")
  ( /opt/rocm/bin/hipcc $F $d -c lean.hip -o /tmp/lean_$n.o && \
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib/libcqgpu_$n.so ../lib/scan.o /tmp/lean_$n.o \
        ../lib/executor.o ../lib/route.o ../lib/prim.o ../lib/writer.o ../lib/merge.o ../lib/hostcell.o ) &
done
wait
