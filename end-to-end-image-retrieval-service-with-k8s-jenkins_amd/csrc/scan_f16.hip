// scan_f16.hip — instantiates the streaming scan + top-k for f16 index rows.
#define SCAN_INSTANTIATE 1
#include "index_common.h"

namespace rc {
void launch_scan_f16(const ScanArgs &a) { launch_scan_dtype<f16_t>(a); }
void launch_query1_f16(const Query1Args &a, hipStream_t s) { launch_query1_dtype<f16_t>(a, s); }
}  // namespace rc
