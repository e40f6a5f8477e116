// sort.hip -- device radix sort of record byte offsets (row-returning SELECT:
// the scan emits matching records in completion order, build_result wants file
// order, evaluator_utils.c:249-549 over filter_rows' row order).
#include <hipcub/hipcub.hpp>

extern "C" hipError_t cq_sort_offsets(void* temp, size_t* temp_bytes, const unsigned long long* in,
                                      unsigned long long* out, size_t n, int bits, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortKeys(temp, *temp_bytes, in, out, (int)n, 0, bits, s);
}
