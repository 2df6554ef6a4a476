// scan_f32.hip — instantiates the streaming scan + top-k for f32 index rows.
#define SCAN_INSTANTIATE 1
#include "index_common.h"

namespace rc {
void launch_scan_f32(const ScanArgs &a) { launch_scan_dtype<float>(a); }
}  // namespace rc
