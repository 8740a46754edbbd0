// ecamd_stream_w8.hip -- gf16_stream_kernel instantiations for 8-output passes.
#include "ecamd_stream.hpp"

ECAMD_STREAM_KG(8, 1, false, false)
ECAMD_STREAM_KG(8, 1, true, false)
ECAMD_STREAM_KG(8, 1, false, true)
ECAMD_PTRS_KG(8)
ECAMD_HYBRID_KG
