# profiling build of libcqgpu.so with per-phase clocks in lean_kernel (-DLEAN_CLK)
set -e
cd "$(dirname "$0")/../cq_amd/csrc"
hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include -DLEAN_CLK -c lean.hip -o /tmp/lean_clk.o 2>/dev/null
hipcc -shared --offload-arch=gfx950 -o ../lib/libcqgpu_clk.so ../lib/scan.o /tmp/lean_clk.o ../lib/executor.o ../lib/sort.o ../lib/hostcell.o
