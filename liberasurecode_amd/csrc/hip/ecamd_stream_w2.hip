// ecamd_stream_w2.hip -- gf16_stream_kernel instantiations for 2-output passes.
#include "ecamd_stream.hpp"

ECAMD_STREAM_KG(2, 1, false, false)
ECAMD_STREAM_KG(2, 1, true, false)
ECAMD_STREAM_KG(2, 1, false, true)
ECAMD_STREAM_KG(2, 2, true, false)
ECAMD_STREAM_KG(2, 2, false, false)
ECAMD_PTRS_KG(2)
ECAMD_REALIGN_KG(2)
