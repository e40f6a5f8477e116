# profiling builds of libcqgpu.so (same sources, parts compiled out or switched)
set -e
cd "$(dirname "$0")/../cq_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include"
b() { name=$1; shift; hipcc $F "$@" -c scan.hip -o /tmp/scan_$name.o && hipcc -shared --offload-arch=gfx950 -o ../lib/libcqgpu_$name.so /tmp/scan_$name.o ../lib/executor.o; }
for v in ${BUILD:-"s0:-DCQ_PROF_STAGE=0" "s1:-DCQ_PROF_STAGE=1" "s1n:-DCQ_PROF_STAGE=1 -DCQ_NO_INDEX" "s2:-DCQ_PROF_STAGE=2"}; do
  b ${v%%:*} ${v#*:} &
done
wait
