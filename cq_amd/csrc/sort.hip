// sort.hip -- device radix sort of record byte offsets (row-returning SELECT:
// the scan emits matching records in completion order, build_result wants file
// order, evaluator_utils.c:249-549 over filter_rows' row order).
#include <hipcub/hipcub.hpp>

extern "C" hipError_t cq_sort_offsets(void* temp, size_t* temp_bytes, const unsigned long long* in,
                                      unsigned long long* out, size_t n, int bits, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortKeys(temp, *temp_bytes, in, out, (int)n, 0, bits, s);
}

// INNER JOIN: right-side key codes with their row indices, stable (equal keys keep
// row order, as the reference's nested loop visits them)
extern "C" hipError_t cq_sort_codes(void* temp, size_t* temp_bytes, const unsigned long long* kin,
                                    unsigned long long* kout, const unsigned int* vin, unsigned int* vout, size_t n,
                                    hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, kin, kout, vin, vout, (int)n, 0, 64, s);
}
// match counts -> pair offsets; pass flags -> output positions
extern "C" hipError_t cq_excl_sum_u64(void* temp, size_t* temp_bytes, const unsigned long long* in,
                                      unsigned long long* out, size_t n, hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, in, out, (int)n, s);
}
extern "C" hipError_t cq_excl_sum_u32(void* temp, size_t* temp_bytes, const unsigned int* in, unsigned int* out,
                                      size_t n, hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, in, out, (int)n, s);
}

// right-side rows grouped by key class (stable: row order within a class)
extern "C" hipError_t cq_sort_classes(void* temp, size_t* temp_bytes, const unsigned int* kin, unsigned int* kout,
                                      const unsigned int* vin, unsigned int* vout, size_t n, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, kin, kout, vin, vout, (int)n, 0, 2, s);
}
// then by key code within each class segment (stable)
extern "C" hipError_t cq_sort_codes_seg(void* temp, size_t* temp_bytes, const unsigned long long* kin,
                                        unsigned long long* kout, const unsigned int* vin, unsigned int* vout,
                                        size_t n, const int* seg_begin, const int* seg_end, int nseg, hipStream_t s) {
    return hipcub::DeviceSegmentedRadixSort::SortPairs(temp, *temp_bytes, kin, kout, vin, vout, (int)n, nseg,
                                                       seg_begin, seg_end, 0, 64, s);
}
