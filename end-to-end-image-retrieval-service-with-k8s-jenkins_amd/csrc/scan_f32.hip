// scan_f32.hip — instantiates the streaming scan + top-k for f32 index rows.
#define SCAN_INSTANTIATE 1
#include "index_common.h"

namespace rc {
void launch_scan_f32(const ScanArgs &a) { launch_scan_dtype<float>(a); }
void launch_query1_f32(const Query1Args &a, hipStream_t s) { launch_query1_dtype<float>(a, s); }
}  // namespace rc
