// hostcell.cpp -- cell.h's typing (parse_value / infer_type restatement) compiled
// for the host, so the executor types SQL literals without a device round trip.
// Same source as the kernels' parser (cell.h), built by g++ without __HIPCC__.
#include <cstring>
#include "cell.h"

extern "C" cq::Cell cq_host_parse_cell(const uint8_t* text, uint32_t len) { return cq::parse_cell(text, len); }
