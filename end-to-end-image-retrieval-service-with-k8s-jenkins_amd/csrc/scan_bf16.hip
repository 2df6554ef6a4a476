// scan_bf16.hip — instantiates the streaming scan + top-k for bf16 index rows.
#define SCAN_INSTANTIATE 1
#include "index_common.h"

namespace rc {
void launch_scan_bf16(const ScanArgs &a) { launch_scan_dtype<bf16_t>(a); }
void launch_query1_bf16(const Query1Args &a, hipStream_t s) { launch_query1_dtype<bf16_t>(a, s); }
}  // namespace rc
