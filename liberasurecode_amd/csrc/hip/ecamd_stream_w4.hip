// ecamd_stream_w4.hip -- gf16_stream_kernel instantiations for 4-output passes.
#include "ecamd_stream.hpp"

ECAMD_STREAM_KG(4, 1, false, false)
ECAMD_STREAM_KG(4, 1, true, false)
ECAMD_STREAM_KG(4, 1, false, true)
ECAMD_STREAM_KG(4, 2, true, false)
ECAMD_STREAM_KG(4, 2, false, false)
ECAMD_PTRS_KG(4)
ECAMD_REALIGN_KG(4)
