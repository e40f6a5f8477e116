# Host-ASan build of libcqgpu's sources + the reference front end + the dense-merge
# driver (scripts/asan_dense.hip), into gpurun_out/asan/ (built here, run on the box):
#   bash scripts/asan_dense.sh build            (in the build container)
#   gpurun_out/asan/asan_dense FILE N "SQL" ... (on the GPU box)
set -e
REF=${REF:-/root/reference}
OUT=${OUT:-asan_build}
mkdir -p $OUT
HF="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -Iinclude"
for f in cq_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  /opt/rocm/bin/hipcc $HF -ffp-contract=off -Wno-unused-value -c $f -o $OUT/$b.o &
done
/opt/rocm/bin/hipcc $HF -c scripts/asan_dense.hip -o $OUT/driver.o &
g++ -O1 -g -std=c++17 -fPIC -fsanitize=address -fno-omit-frame-pointer -c cq_amd/csrc/hostcell.cpp -o $OUT/hostcell.o &
wait
for f in $REF/src/tokenizer.c $REF/src/parser.c $REF/src/parser/*.c $REF/src/utils.c $REF/src/csv_reader.c $REF/src/date_utils.c $REF/src/mmap.c; do
  gcc -O1 -g -w -fsanitize=address -fno-omit-frame-pointer -I$REF/include -c $f -o $OUT/ref_$(basename $f .c).o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fsanitize=address -o $OUT/asan_dense $OUT/*.o -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
